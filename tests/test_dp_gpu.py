"""Data-parallel step on a real GPU through RCCL (single-rank process group): the bucketed
all-reduce path of hpnn_amd.parallel.DataParallel must give the same weights as the plain
single-GPU step (an all-reduce over one rank is the identity)."""
import pytest
import torch
import torch.distributed as dist

from hpnn_amd.models import MLP
from hpnn_amd.parallel import DataParallel


@pytest.mark.gpu
@pytest.mark.parametrize("comm", ["native", "torch"])
@pytest.mark.parametrize("sizes", [[784, 128, 64, 10], [300, 96, 40, 7]])
def test_dp_rccl_single_rank_matches_plain(gpu, sizes, comm):
    dev = torch.device("cuda", 0)
    store = dist.HashStore()
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        g = torch.Generator(device=dev).manual_seed(7)
        B = 4096
        Xr = torch.rand(B, sizes[0], device=dev, generator=g)
        L = torch.randint(0, sizes[-1], (B,), device=dev, generator=g, dtype=torch.int32)
        a = MLP(sizes, "SNN", batch=B, device=dev, momentum=True, seed=3)
        b = MLP(sizes, "SNN", batch=B, device=dev, momentum=True, seed=3)
        dp = DataParallel(a, comm=comm)
        assert dp.active and dp.world == 1
        assert (dp.native is not None) == (comm == "native")
        Xa, Xb = a.prepare_input(Xr), b.prepare_input(Xr)
        for _ in range(3):
            dp.train_step(Xa, labels=L, lr=0.05, alpha=0.2)
            b.train_step(Xb, labels=L, lr=0.05, alpha=0.2)
        torch.cuda.synchronize()
        for wa, wb in zip(a.host_weights(), b.host_weights()):
            # same math; the fused single-GPU step sums the split-K slabs in a different order
            assert (wa - wb).abs().max().item() < 1e-6
        assert dp.all_ok(True)
        dp.check()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_native_comm_primitives_single_rank(gpu):
    """libhpnn's RCCL communicator (csrc/dist/comm.cpp) on a one-rank group: every
    collective is the identity, async all-reduce + join are ordered on the stream, the
    status agreement and the error check work, and an injected fault surfaces."""
    from hpnn_amd._lib import native
    from hpnn_amd.parallel import NativeComm
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    try:
        c = NativeComm()
        assert (c.rank, c.world) == (0, 1)
        x = torch.arange(1000, dtype=torch.float32, device=dev)
        ref = x.clone()
        c.all_reduce(x)
        c.broadcast(x, root=0)
        out = torch.empty_like(x)
        c.all_gather(out, x)
        rs = torch.empty_like(x)
        c.reduce_scatter(rs, x)
        y = torch.ones(4096, device=dev)
        y.mul_(3.0)
        c.all_reduce_async(y)
        c.join()
        y.add_(1.0)  # ordered after the joined all-reduce
        torch.cuda.synchronize()
        assert torch.equal(x, ref) and torch.equal(out, ref) and torch.equal(rs, ref)
        assert torch.equal(y, torch.full_like(y, 4.0))
        for dt in (torch.float64, torch.bfloat16, torch.int32):
            z = torch.arange(64, device=dev).to(dt)
            c.all_reduce(z)
            assert torch.equal(z.cpu(), torch.arange(64).to(dt))
        assert c.all_ok(True) and not c.all_ok(False)
        c.check()
        c.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("grad_comm,sizes", [("fp32", [300, 96, 64, 7]), ("bf16rs", [300, 96, 64, 7]),
                                             ("bf16rs", [1024, 512, 256, 10])])
def test_native_dp_exchange_single_rank(gpu, monkeypatch, grad_comm, sizes):
    """the library's data-parallel step (csrc/dist/dp_exchange.cpp, hpnn::DpExchange) forced
    onto a one-rank RCCL group (HPNN_DPX_FORCE / HPNN_DPX_SHARD1): fp32 = per-layer bucket
    all-reduce on the communicator's side stream + one update; bf16rs = per-layer BF16 cast ->
    reduce-scatter -> row step of the FP32 masters -> in-place BF16 all-gather -> W^T rebuild.
    Against the plain step: fp32 to summation order, bf16rs within the BF16 rounding of the
    gradient (relative error of the weight change < 1e-2).  [1024, 512, 256, 10]: layer 1's delta
    GEMM reads the all-gathered W (NN form) and skips the W^T rebuild; gather_masters makes W^T
    current again."""
    monkeypatch.setenv("HPNN_DPX_FORCE", "1")
    monkeypatch.setenv("HPNN_DPX_SHARD1", "1")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    try:
        B = 2048
        g = torch.Generator(device=dev).manual_seed(5)
        Xr = torch.rand(B, sizes[0], device=dev, generator=g)
        L = torch.randint(0, sizes[-1], (B,), device=dev, generator=g, dtype=torch.int32)
        a = MLP(sizes, "SNN", batch=B, device=dev, momentum=True, seed=3, fused=False)
        b = MLP(sizes, "SNN", batch=B, device=dev, momentum=True, seed=3, fused=False)
        w0 = [w.clone() for w in b.host_weights()]
        dp = DataParallel(a, comm="native", grad_comm=grad_comm)
        assert dp.dpx is not None
        if grad_comm == "bf16rs":
            assert dp.sharded == set(range(3))
            assert list(a.plan.nn_bwd[:3]) == ([False, True, False] if sizes[0] == 1024 else [False] * 3)
        Xa, Xb = a.prepare_input(Xr), b.prepare_input(Xr)
        for _ in range(3):
            dp.train_step(Xa, labels=L, lr=0.05, alpha=0.2)
            b.train_step(Xb, labels=L, lr=0.05, alpha=0.2)
        dp.gather_masters()
        torch.cuda.synchronize()
        for l, (wa, wb) in enumerate(zip(a.host_weights(), b.host_weights())):
            da, db = wa - w0[l], wb - w0[l]
            rel = ((da - db).norm() / db.norm()).item()
            assert rel < (1e-5 if grad_comm == "fp32" else 1e-2), (l, rel)
            # the BF16 compute copies follow the masters
            assert torch.equal(a.Wb[l], a.W32[l].bfloat16())
            assert torch.equal(a.Wt[l], a.W32[l].bfloat16().t().contiguous())
        dp.check()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_native_dp_exchange_emulated_world(gpu, monkeypatch):
    """HPNN_DPX_EMULATE_WORLD=8 on one rank (csrc/dist/dp_exchange.cpp): the sharded BF16 step
    at 8-rank sizes -- rank 0's 1/8 of every layer's rows reduce-scattered (a copy on one rank)
    and stepped, the all-gather's receive bytes copied locally.  Those rows follow the plain
    step within the BF16 rounding of the gradient; every other row keeps its initial master
    (the timing knob for the per-rank compute of the 8-GPU strong-scaling shard)."""
    monkeypatch.setenv("HPNN_DPX_FORCE", "1")
    monkeypatch.setenv("HPNN_DPX_EMULATE_WORLD", "8")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    try:
        sizes, B = [2048, 1024, 512, 64], 1024
        g = torch.Generator(device=dev).manual_seed(6)
        Xr = torch.rand(B, sizes[0], device=dev, generator=g)
        L = torch.randint(0, sizes[-1], (B,), device=dev, generator=g, dtype=torch.int32)
        a = MLP(sizes, "SNN", batch=B, device=dev, momentum=True, seed=3, fused=False)
        b = MLP(sizes, "SNN", batch=B, device=dev, momentum=True, seed=3, fused=False)
        w0 = [w.clone() for w in a.W32]
        dp = DataParallel(a, comm="native", grad_comm="bf16rs")
        assert dp.dpx is not None and dp.sharded == set(range(3))
        dp.train_step(a.prepare_input(Xr), labels=L, lr=0.05, alpha=0.2)
        b.train_step(b.prepare_input(Xr), labels=L, lr=0.05, alpha=0.2)
        dp.gather_masters()  # nothing to gather; W^T of the NN-form layers made current
        torch.cuda.synchronize()
        assert list(a.plan.nn_bwd[:3]) == [False, True, True]
        for l in range(3):
            assert torch.equal(a.Wt[l], a.W32[l].bfloat16().t()), l
            r = a.W32[l].shape[0] // 8
            da, db = a.W32[l][:r] - w0[l][:r], b.W32[l][:r] - w0[l][:r]
            rel = ((da - db).norm() / db.norm()).item()
            assert rel < 1e-2, (l, rel)
            assert torch.equal(a.W32[l][r:], w0[l][r:]), l
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("sizes,expect", [([2048, 1024, 10], "bf16rs"), ([300, 96, 64, 7], "fp32"),
                                          ([4096, 4096, 32], "bf16rs")])
def test_native_dp_exchange_auto_default(gpu, monkeypatch, sizes, expect):
    """grad_comm defaults to "auto": a per-layer net with more than 4 MB of FP32 gradients takes
    the BF16 reduce-scatter + sharded step on the N > 1 path (here one rank, HPNN_DPX_FORCE);
    small ones the FP32 all-reduce.  Both train like the plain step (bf16rs within the BF16
    rounding of the gradient).  4096 x 4096 at batch 1024 is one 8-phase TN split: its GEMM
    writes the BF16 gradient the exchange sends (gemm_tn8_kernel<3>, BPlan::g16)."""
    monkeypatch.setenv("HPNN_DPX_FORCE", "1")
    monkeypatch.setenv("HPNN_DPX_SHARD1", "1")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    try:
        B = 1024
        g = torch.Generator(device=dev).manual_seed(5)
        Xr = torch.rand(B, sizes[0], device=dev, generator=g)
        L = torch.randint(0, sizes[-1], (B,), device=dev, generator=g, dtype=torch.int32)
        init = "fast" if sizes[0] * sizes[1] > 1 << 22 else "reference"
        a = MLP(sizes, "SNN", batch=B, device=dev, momentum=True, seed=3, fused=False, init=init)
        b = MLP(sizes, "SNN", batch=B, device=dev, momentum=True, seed=3, fused=False, init=init)
        w0 = [w.clone() for w in b.host_weights()]
        dp = DataParallel(a, comm="native")
        assert dp.grad_comm == expect and bool(dp.sharded) == (expect == "bf16rs")
        Xa, Xb = a.prepare_input(Xr), b.prepare_input(Xr)
        for _ in range(2):
            dp.train_step(Xa, labels=L, lr=0.05, alpha=0.2)
            b.train_step(Xb, labels=L, lr=0.05, alpha=0.2)
        dp.gather_masters()
        torch.cuda.synchronize()
        for l, (wa, wb) in enumerate(zip(a.host_weights(), b.host_weights())):
            da, db = wa - w0[l], wb - w0[l]
            rel = ((da - db).norm() / db.norm()).item()
            assert rel < (1e-5 if expect == "fp32" else 1e-2), (l, rel)
        dp.check()
    finally:
        dist.destroy_process_group()
