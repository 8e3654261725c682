"""The data-parallel MNIST step on the one-shot xGMI all-reduce with two real processes
(both on the box's single MI355X; RCCL refuses two ranks on one device, so the ranks run
the xGMI-only communicator, comm="xar").  This is the exact step bench.py runs at N > 1:
fused front, G0 GEMM with the [G1|G2] reduction on its tail workgroups, ONE all-reduce
that also sums the local split-K slabs, the update.  Checked: both ranks end with
bit-identical weights, equal (to FP32 summation order) to one process training on the
concatenated batch; a HIP-graph-captured step gives the same result as eager steps."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SIZES = [784, 128, 64, 10]
B = 8192


def _data(rank, step, u8=False, B=B):
    g = torch.Generator().manual_seed(100 * rank + step)
    x = (torch.randint(0, 256, (B, SIZES[0]), generator=g, dtype=torch.uint8) if u8
         else torch.rand(B, SIZES[0], generator=g))
    return x, torch.randint(0, 10, (B,), generator=g, dtype=torch.int32)


def _worker(rank, world, port, graph, q, u8=False, xar_mode=None, form="kernel", B=B, g0_mode=None, perm=0):
    try:
        if g0_mode is not None:  # in-kernel exchange: 1 one-shot, 2 two-shot (auto: two-shot from 4 ranks)
            os.environ["HPNN_XAR_G0_MODE"] = str(g0_mode)
        os.environ["LOCAL_WORLD_SIZE"] = str(world)
        os.environ["HPNN_XAR_G0"] = "1" if form == "kernel" else "0"
        os.environ["HPNN_XAR_LOCAL"] = "1" if form == "buffer" else "0"
        if xar_mode is not None:  # 1 one-shot, 2 two-shot (the default from 4 ranks), unset: auto
            os.environ["HPNN_XAR_MODE"] = str(xar_mode)
        os.environ["HPNN_XAR_TIMEOUT_MS"] = "2000"
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        from hpnn_amd.models import MLP
        from hpnn_amd.parallel import DataParallel
        dev = torch.device("cuda", 0)
        # the ranks share this one GPU and a rank's G0 spins at its exchange barriers until every
        # peer's G0 arrives: every rank's G0 grid must fit on the CUs at once (10 tiles x splits
        # workgroups each, <= 160 together); one GPU per rank in real runs
        m = MLP(SIZES, "SNN", batch=B, device=dev, momentum=True, seed=3, splits=[max(1, 16 // world), 0, 0])
        dp = DataParallel(m, comm="xar")
        m.plan.g0_perm = perm  # > 0: the G0 grid in another block -> role order (same on every rank)
        if form == "kernel":  # the in-kernel exchange needs the fused G0 (tile or fused-x path)
            assert m.fused_mode in ("t", "x") and dp.xar_k, (m.fused_mode, dp.xar_k)
            # DataParallel ran the in-kernel exchange's self-test at attach; once more, checked here
            # (collective: every rank calls it)
            rc = m.plan.xchg_self_test(dp.xar_k, torch.cuda.current_stream().cuda_stream)
            assert rc == 0, rc
        assert dp.native is not None and dp.native.xar and m.fused_mode in ("x", "t")
        dp.broadcast_parameters()
        batches = []
        for step in range(3):
            x, lab = _data(rank, step, u8, B)
            batches.append((m.prepare_input(x.to(dev)), lab.to(dev)))
            if u8:  # 8-bit pixels: fragment-major byte copy for the first-layer gradient
                assert m._fm_input(batches[-1][0]) is not None
        if graph:
            # step 0 eager, steps 1-2 from one captured graph replayed twice over the same inputs
            dp.train_step(batches[0][0], labels=batches[0][1], lr=0.05, alpha=0.2)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                with torch.cuda.graph(g):
                    dp.train_step(batches[1][0], labels=batches[1][1], lr=0.05, alpha=0.2)
            torch.cuda.current_stream().wait_stream(s)
            g.replay()
            g.replay()
        else:
            for step in (0, 1, 1):
                dp.train_step(batches[step][0], labels=batches[step][1], lr=0.05, alpha=0.2)
        torch.cuda.synchronize()
        dp.check()
        # kernel: the exchange ran inside the G0 launch; buffer: the G0 launch wrote the
        # gradient into the all-reduce's buffer half; copy: the all-reduce copied it in
        assert dp.xar_inplace == (form if form != "copy" else False), (dp.xar_inplace, form)
        W = torch.cat([w.flatten() for w in m.W32] + [v.flatten() for v in m.V32]).cpu()
        q.put((rank, W))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))


def _reference(u8=False, world=2, B=B):
    from hpnn_amd.models import MLP
    dev = torch.device("cuda", 0)
    m = MLP(SIZES, "SNN", batch=world * B, device=dev, momentum=True, seed=3)
    for step in (0, 1, 1):
        xs, ls = zip(*[_data(r, step, u8, B) for r in range(world)])
        X = m.prepare_input(torch.cat(xs).to(dev))
        m.train_step(X, labels=torch.cat(ls).to(dev), lr=0.05, alpha=0.2)
    torch.cuda.synchronize()
    return torch.cat([w.flatten() for w in m.W32] + [v.flatten() for v in m.V32]).cpu()


def _run(world, graph, u8, xar_mode=None, form="kernel", B=B, g0_mode=None, perm=0, check_ref=True):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, graph, q, u8, xar_mode, form, B, g0_mode, perm))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=110 if world <= 2 else 250) for _ in ps)
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    for r in range(world):
        assert isinstance(res[r], torch.Tensor), res[r]
    for r in range(1, world):
        assert torch.equal(res[0], res[r])  # deterministic, identical on every rank
    if check_ref:
        ref = _reference(u8, world, B)
        err = (res[0] - ref).abs().max().item()
        assert err < 2e-6, err
    return res[0]


@pytest.mark.gpu
@pytest.mark.parametrize("graph,u8", [(False, False), (True, False), (True, True)])
def test_dp_step_on_xgmi_allreduce_two_processes(gpu, graph, u8):
    _run(2, graph, u8)


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["buffer", "copy"])
def test_dp_step_separate_exchange_forms(gpu, form):
    """HPNN_XAR_G0=0: the exchange in its own launch after the G0 launch, which writes the
    all-reduce's buffer half (buffer) or the plan's gradient buffer for the all-reduce to
    copy in (copy, HPNN_XAR_LOCAL=0): same weights as the in-kernel exchange"""
    _run(2, True, False, None, form)


@pytest.mark.gpu
def test_dp_step_two_shot_with_fused_update(gpu):
    """the two-shot all-reduce with the optimizer step fused in (each rank updates its own
    shard in the reduce phase and the peers' shards after the gather), forced at 2 ranks in
    the whole DP step.  (3+ ranks of the full step cannot share ONE GPU: a rank's fused
    front kernel needs whole CUs while the other ranks' all-reduce workgroups spin on
    theirs; the two-shot + update exchange itself runs at 3, 4 and 8 ranks in
    tests/test_xar_gpu.py.)"""
    _run(2, True, True, 2, "buffer")


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,batch,g0_mode", [(4, 4096, None), (8, 2048, None), (4, 4096, 1), (8, 2048, 1)])
def test_dp_step_in_kernel_exchange_many_ranks(gpu, world, batch, g0_mode):
    """the in-kernel exchange (flag barriers per G0 workgroup with every peer) at 4 and 8 ranks,
    two-shot (the default from 4 ranks) and one-shot, graph-captured, 8-bit input.  The ranks
    share this one GPU, so every rank's G0 grid (10 tiles x 16 / world splits) plus its front
    must fit on the CUs at once: a rank's G0 spins at its barriers until every peer's G0
    arrives."""
    _run(world, True, True, None, "kernel", batch, g0_mode)


@pytest.mark.gpu
def test_dp_step_in_kernel_exchange_two_shot_two_ranks(gpu):
    """the two-shot in-kernel exchange forced at 2 ranks (HPNN_XAR_G0_MODE=2)"""
    _run(2, True, True, None, "kernel", B, 2)


@pytest.mark.gpu
def test_dp_step_in_kernel_exchange_fused_x_mode(gpu):
    """a per-rank batch that is not a whole number of 256-sample tiles (8320 = 65 x 128) runs
    the fused-x front (kernels_mlp3x.hip) before the same G0 launch with the exchange"""
    _run(2, True, True, None, "kernel", 8320)


@pytest.mark.gpu
def test_in_kernel_exchange_role_order_bitwise(gpu):
    """the in-kernel exchange's results do not depend on which workgroup takes which role
    (tile, split, exchange slot): the G0 grid run in reversed / rotated block orders gives
    bitwise the same weights (every sum has a fixed order; the block -> XCD placement is a
    speed assumption only)"""
    base = _run(2, True, True, check_ref=False)
    for perm in (80, 37):  # 80 = the reversed order (80 workgroups a rank), 37: reversed + rotated
        assert torch.equal(_run(2, True, True, perm=perm, check_ref=False), base), perm
