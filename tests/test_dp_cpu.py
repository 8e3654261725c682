"""Data parallel over torch.distributed (gloo, 2 CPU ranks) == one process on the whole
batch.  Exercises the bucketing / all-reduce / update orchestration of
hpnn_amd.parallel.DataParallel with the PyTorch emulation of the kernels (CPU tensors)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hpnn_amd.models import MLP
from hpnn_amd.parallel import DataParallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sizes, net, fused, B, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    Xall = torch.rand(B * world, sizes[0])
    Lall = torch.randint(0, sizes[-1], (B * world,), dtype=torch.int32)
    m = MLP(sizes, net, batch=B, device="cpu", momentum=True, seed=11, fused=fused)
    dp = DataParallel(m, bucket_bytes=16 * 1024)
    dp.broadcast_parameters()
    X = m.prepare_input(Xall[rank * B:(rank + 1) * B])
    L = Lall[rank * B:(rank + 1) * B]
    for _ in range(steps):
        dp.train_step(X, labels=L, lr=0.05, alpha=0.2)
    # the replica digest is process-independent: identical replicas agree across processes
    ok = dp.weights_consistent()
    if rank == 0:
        q.put((ok, [w.numpy() for w in m.host_weights()]))  # by value: no shared-memory fd
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sizes,net,fused", [([32, 128, 64, 10], "SNN", True), ([32, 128, 64, 10], "SNN", False),
                                             ([16, 24, 5], "ANN", False)])
def test_dp_equals_single(sizes, net, fused):
    world, B, steps = 2, 128, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sizes, net, fused, B, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok, got = q.get(timeout=300)
    assert ok, "weights_consistent() disagrees for identical CPU replicas"
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    torch.manual_seed(0)
    Xall = torch.rand(B * world, sizes[0])
    Lall = torch.randint(0, sizes[-1], (B * world,), dtype=torch.int32)
    m = MLP(sizes, net, batch=B * world, device="cpu", momentum=True, seed=11, fused=fused)
    X = m.prepare_input(Xall)
    for _ in range(steps):
        m.train_step(X, labels=Lall, lr=0.05, alpha=0.2)
    for a, b in zip(got, m.host_weights()):
        a = torch.as_tensor(a)
        assert (a - b).abs().max().item() < 1e-5, (a - b).abs().max().item()


def test_bucket_plan():
    m = MLP([784, 128, 64, 10], "SNN", batch=128, device="cpu")
    dp = DataParallel(m, bucket_bytes=64 * 1024)
    flat = [l for b in dp.buckets for l in b]
    assert sorted(flat) == [0, 1, 2] and dp.buckets[0][0] == 2
    for b in dp.buckets:
        v = dp._bucket_view(b)
        assert v.numel() == sum(m.G[l].numel() for l in b)


def test_split_counts_for_8phase_tn():
    """weight gradients with 256x256 tiles get a split count the 8-phase TN kernel accepts
    (>= 256 workgroups, an even number of 64-row units per split); others keep the
    one-workgroup-per-CU rule (MNIST's G0: 48).  One rule, in the library (bplan.cpp)."""
    from hpnn_amd.models.mlp import MLP
    assert MLP._pick_splits(256, 4096, 16384) == 16       # RRUFF-shaped first layer
    assert MLP._pick_splits(4096, 4096, 8192) == 1        # synthetic 8x4096 ANN
    assert MLP._pick_splits(128, 800, 65536) == 48        # MNIST G0 (not 256-divisible)
    for N, K, B in [(256, 4096, 16384), (512, 2048, 8192), (4096, 4096, 1024)]:
        s = MLP._pick_splits(N, K, B)
        assert (N // 256) * (K // 256) * s >= 256 and (B // 64) % s == 0 and (B // 64 // s) % 2 == 0
    assert MLP._pick_splits(256, 256, 16384) == 32        # no 8-phase split: 32 splits of 512 rows


def _worker_rs(rank, world, port, sizes, B, steps, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    Xall = torch.rand(B * world, sizes[0])
    Lall = torch.randint(0, sizes[-1], (B * world,), dtype=torch.int32)
    m = MLP(sizes, "ANN", batch=B, device="cpu", momentum=True, seed=11, fused=False)
    dp = DataParallel(m, grad_comm=mode)
    dp.broadcast_parameters()
    T = torch.full((B * world, sizes[-1]), -1.0)
    T[torch.arange(B * world), Lall.long()] = 1.0
    X = m.prepare_input(Xall[rank * B:(rank + 1) * B])
    for _ in range(steps):
        dp.train_step(X, T=T[rank * B:(rank + 1) * B], lr=0.05, alpha=0.2)
    if mode == "bf16rs":
        assert dp.sharded == {0, 1, 2}  # padded rows (64, 32, 32) split evenly over 2 ranks
        dp.gather_masters()
    q.put((rank, [w.numpy() for w in m.host_weights()], [b.float().numpy() for b in m.Wb]))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_bf16_reduce_scatter_sharded_update():
    """grad_comm='bf16rs': BF16 reduce-scatter, each rank steps its rows of the FP32
    masters, BF16 weights all-gathered -> identical BF16 weights on every rank, and the
    same training as the FP32 all-reduce up to the BF16 rounding of the gradient sum."""
    world, B, steps, sizes = 2, 128, 3, [24, 64, 32, 5]
    res = {}
    for mode in ("fp32", "bf16rs"):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_worker_rs, args=(r, world, port, sizes, B, steps, mode, q)) for r in range(world)]
        for p in procs:
            p.start()
        got = {r: ([torch.as_tensor(x) for x in w], [torch.as_tensor(x) for x in b])
               for r, w, b in (q.get(timeout=120) for _ in procs)}
        for p in procs:
            p.join(timeout=300)
            assert p.exitcode == 0
        res[mode] = got
    rs = res["bf16rs"]
    for a, b in zip(rs[0][0], rs[1][0]):
        assert torch.equal(a, b)  # gathered masters identical
    for a, b in zip(rs[0][1], rs[1][1]):
        assert torch.equal(a, b)  # BF16 compute weights identical on every rank
    W0 = MLP(sizes, "ANN", batch=B, device="cpu", seed=11).host_weights()
    for w0, a, b in zip(W0, rs[0][0], res["fp32"][0][0]):
        da, db = a - w0, b - w0
        rel = (da - db).norm() / (db.norm() + 1e-30)
        assert rel < 2e-2, rel.item()


def _worker_auto(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    for name, sizes, fused in (("big", [1100, 1024, 10], False), ("small", [24, 64, 32, 5], False),
                               ("mnist", [784, 128, 64, 10], None)):
        m = MLP(sizes, "SNN", batch=128, device="cpu", seed=11, fused=fused)
        dp = DataParallel(m)  # grad_comm="auto"
        out[name] = (dp.grad_comm, sorted(dp.sharded))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_grad_comm_auto():
    """grad_comm="auto" (the default): the BF16 reduce-scatter + sharded update for per-layer
    models whose FP32 gradients exceed 4 MB at world > 1; the FP32 all-reduce otherwise
    (small gradients are latency-bound, and the fused MNIST-shape step exchanges in-kernel)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_auto, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in range(world):
        assert got[r]["big"] == ("bf16rs", [0, 1])
        assert got[r]["small"] == ("fp32", [])
        assert got[r]["mnist"] == ("fp32", [])
    # one rank: nothing to exchange, the plain path
    m = MLP([1100, 1024, 10], "SNN", batch=128, device="cpu", fused=False)
    assert DataParallel(m).grad_comm == "fp32"
