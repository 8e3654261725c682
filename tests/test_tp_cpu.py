"""Row-sharded tensor parallelism (gloo, 2 CPU ranks) == single-process training."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hpnn_amd.models import MLP
from hpnn_amd.parallel import TensorParallelMLP


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sizes, net, B, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    X = torch.rand(B, sizes[0])
    L = torch.randint(0, sizes[-1], (B,), dtype=torch.int32)
    tp = TensorParallelMLP(sizes, net, batch=B, device="cpu", momentum=True, seed=21)
    Xp = torch.zeros(tp.Bp, tp.Kp[0], dtype=torch.bfloat16)
    Xp[:B, :sizes[0]] = X.bfloat16()
    for _ in range(steps):
        tp.train_step(Xp, labels=L, lr=0.05, alpha=0.2)
    w = tp.full_weights()
    if rank == 0:
        q.put([t.numpy() for t in w])  # by value: no shared-memory fd to outlive the child
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sizes,net", [([40, 96, 64, 10], "SNN"), ([24, 50, 7], "ANN")])
def test_tp_equals_single(sizes, net):
    world, B, steps = 2, 128, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, sizes, net, B, steps, q)) for r in range(world)]
    for p in ps:
        p.start()
    import queue
    try:
        got = q.get(timeout=120)
    except queue.Empty:
        for p in ps:
            p.kill()
        raise
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0
    torch.manual_seed(0)
    X = torch.rand(B, sizes[0])
    L = torch.randint(0, sizes[-1], (B,), dtype=torch.int32)
    m = MLP(sizes, net, batch=B, device="cpu", momentum=True, seed=21, fused=False)
    Xd = m.prepare_input(X)
    for _ in range(steps):
        m.train_step(Xd, labels=L, lr=0.05, alpha=0.2)
    for a, b in zip(got, m.host_weights()):
        a = torch.as_tensor(a)
        assert (a - b).abs().max().item() < 1e-4, (a - b).abs().max().item()
