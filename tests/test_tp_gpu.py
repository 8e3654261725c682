"""Row-sharded tensor parallelism on the GPU kernels with two processes sharing the box's
one MI355X (gloo carries the activation all-gathers and partial-delta reduce-scatters
through host memory; RCCL refuses two ranks on one device): every step on the native
kernels (gemm_nt / block_permute / dact_cast / gemm_tn / sgd_update_multi) == single-process
GPU training."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SIZES = [200, 96, 64, 10]
B = 1024


def _inputs():
    g = torch.Generator().manual_seed(0)
    return torch.rand(B, SIZES[0], generator=g), torch.randint(0, SIZES[-1], (B,), generator=g, dtype=torch.int32)


def _worker(rank, world, port, q):
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        from hpnn_amd.parallel import TensorParallelMLP
        dev = torch.device("cuda", 0)
        X, L = _inputs()
        tp = TensorParallelMLP(SIZES, "SNN", batch=B, device=dev, momentum=True, seed=21)
        Xp = torch.zeros(tp.Bp, tp.Kp[0], dtype=torch.bfloat16, device=dev)
        Xp[:B, :SIZES[0]] = X.to(dev).bfloat16()
        for _ in range(3):
            tp.train_step(Xp, labels=L.to(dev), lr=0.05, alpha=0.2)
        w = tp.full_weights()
        q.put((rank, w))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.gpu
def test_tp_two_processes_on_gpu_equals_single(gpu):
    from hpnn_amd.models import MLP
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=110) for _ in ps)
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert isinstance(res[0], list), res[0]
    assert isinstance(res[1], list), res[1]
    dev = torch.device("cuda", 0)
    X, L = _inputs()
    m = MLP(SIZES, "SNN", batch=B, device=dev, momentum=True, seed=21, fused=False)
    Xm = m.prepare_input(X.to(dev))
    for _ in range(3):
        m.train_step(Xm, labels=L.to(dev), lr=0.05, alpha=0.2)
    torch.cuda.synchronize()
    for a, b, ref in zip(res[0], res[1], m.host_weights()):
        assert torch.equal(a, b)
        assert (a - ref).abs().max().item() < 2e-3, (a - ref).abs().max().item()
