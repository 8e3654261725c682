"""xGMI all-reduce (csrc/dist/xgmi_ar.hip), one-shot and two-shot, with 2-4 real processes.

The GPU box has one MI355X, so both ranks run on device 0: the peer buffers are mapped
through hipIpc exactly as on an 8-GPU node (the data path is then local HBM instead of
an xGMI link, the protocol -- IPC mapping, flag barriers, epochs, fixed-order sum -- is
the same).  Checked: sums of several bucket sizes against the host sum, in-place use,
the attach-time self-test, repeated calls (alternating buffer halves, mixed one-/two-shot calls in auto mode at 4
ranks), slab-sum inputs, HIP-graph capture + replays, and the bounded barrier: a rank
whose peer never arrives reports a timeout instead of hanging."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SIZES = [4, 1024, 9280, 102400, 262144]


def _data(rank, n, it):
    g = torch.Generator().manual_seed(1000 * rank + 7 * it + n)
    return torch.randn(n, generator=g)


def _check_slabs_update(n, x, rank, world, s):
    """the all-reduce with every layer's optimizer step fused in (the DP MNIST step's
    exchange): MNIST-shaped layers (G0 128 x 800 from 3 split-K slabs, [G1 | G2] from 2
    group slabs, 450 KB: two-shot from 4 ranks in auto mode), BPM; every rank must end with
    the same W32 / V32 / BF16 copies as a host update on the summed gradient"""
    shapes = [(128, 800), (64, 128), (32, 64)]
    lr, alpha, scale = 0.05, 0.2, 1.0 / 777
    g = torch.Generator().manual_seed(5)  # same initial weights on every rank
    Ws = [torch.randn(N, K, generator=g) * 0.1 for N, K in shapes]
    Vs = [torch.randn(N, K, generator=g) * 0.01 for N, K in shapes]
    W32 = [w.clone().cuda() for w in Ws]
    V32 = [v.clone().cuda() for v in Vs]
    Wb = [torch.empty(N, K, dtype=torch.bfloat16, device="cuda") for N, K in shapes]
    Wt = [torch.empty(K, N, dtype=torch.bfloat16, device="cuda") for N, K in shapes]
    n0 = 128 * 800
    n12 = 64 * 128 + 32 * 64
    sl0 = torch.stack([_data(rank, n0, 200 + k) for k in range(3)]).cuda()
    sl1 = torch.stack([_data(rank, n12, 300 + k) for k in range(2)]).cuda()
    out = torch.empty(n0 + n12, device="cuda")
    layers = [(W32[i].data_ptr(), V32[i].data_ptr(), Wb[i].data_ptr(), Wt[i].data_ptr(), 0, N, K)
              for i, (N, K) in enumerate(shapes)]
    n.xar_all_reduce_slabs_update_f32(x, [(sl0.data_ptr(), sl0.stride(0), 3, n0), (sl1.data_ptr(), sl1.stride(0), 2,
                                                                                    n12)],
                                      out.data_ptr(), layers, lr, alpha, scale, 1, s)
    torch.cuda.synchronize()
    G = torch.cat([sum(_data(r, n0, 200 + k) for r in range(world) for k in range(3)),
                   sum(_data(r, n12, 300 + k) for r in range(world) for k in range(2))])
    errs = []
    if (out.cpu() - G).abs().max().item() > 1e-4:
        errs.append("slabs-update: reduced gradient mismatch")
    off = 0
    for i, (N, K) in enumerate(shapes):
        gi = G[off:off + N * K].view(N, K) * scale
        off += N * K
        v = Vs[i] + lr * gi
        w = Ws[i] + v
        v = v * alpha
        if (W32[i].cpu() - w).abs().max().item() > 1e-5 or (V32[i].cpu() - v).abs().max().item() > 1e-6:
            errs.append(f"slabs-update: layer {i} W32/V32 mismatch")
        if not torch.equal(Wb[i].cpu(), W32[i].cpu().bfloat16()) or not torch.equal(Wt[i].cpu(),
                                                                                     W32[i].cpu().bfloat16().t()):
            errs.append(f"slabs-update: layer {i} bf16 copies mismatch")
    return errs


def _worker(rank, world, port, q, mode):
    try:
        os.environ["HPNN_XAR_TIMEOUT_MS"] = "400"
        os.environ["HPNN_XAR_MODE"] = mode
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        from hpnn_amd._lib import native
        n = native()
        x = n.xar_create(rank, world, 1 << 20)
        assert x
        h = torch.tensor(list(n.xar_handles(x)), dtype=torch.uint8)
        allh = torch.zeros(world * n.XAR_HANDLE_BYTES, dtype=torch.uint8)
        dist.all_gather_into_tensor(allh, h)
        n.xar_open(x, bytes(allh.tolist()))
        dist.barrier()
        s = torch.cuda.current_stream().cuda_stream
        errs = []
        # the attach-time self-test (known exact sums at a one-shot and the full size)
        rc = n.xar_self_test(x, s)
        if rc != 0:
            errs.append(f"self-test returned {rc}")
        for it in range(3):
            for sz in SIZES:
                a = _data(rank, sz, it).cuda()
                out = torch.empty_like(a)
                n.xar_all_reduce_f32(x, a.data_ptr(), out.data_ptr(), sz, s)
                n.xar_all_reduce_f32(x, a.data_ptr(), a.data_ptr(), sz, s)  # in place
                torch.cuda.synchronize()
                ref = sum(_data(r, sz, it) for r in range(world))
                if not torch.equal(out.cpu(), a.cpu()):
                    errs.append(f"in-place != out-of-place size {sz}")
                e = (out.cpu() - ref).abs().max().item()
                if e > 1e-5:
                    errs.append(f"size {sz} it {it}: max err {e}")
        # slab inputs: out = sum over ranks of [sum of 3 slabs of seg 0 | seg 1 (1 slab)]
        sl = torch.stack([_data(rank, 4096, 50 + k) for k in range(3)]).cuda()
        tl = _data(rank, 1000, 60).cuda()
        out = torch.empty(5096, device="cuda")
        n.xar_all_reduce_slabs_f32(x, [(sl.data_ptr(), sl.stride(0), 3, 4096), (tl.data_ptr(), 0, 1, 1000)],
                                   out.data_ptr(), s)
        torch.cuda.synchronize()
        ref = torch.cat([sum(_data(r, 4096, 50 + k) for r in range(world) for k in range(3)),
                         sum(_data(r, 1000, 60) for r in range(world))])
        if (out.cpu() - ref).abs().max().item() > 1e-4:
            errs.append("slab-sum all-reduce mismatch")
        errs += _check_slabs_update(n, x, rank, world, s)
        # graph capture: the kernel advances its own barrier epochs on every replay
        buf = _data(rank, 9280, 99).cuda()
        base = buf.clone()
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            with torch.cuda.graph(g):
                buf.copy_(base)
                n.xar_all_reduce_f32(x, buf.data_ptr(), buf.data_ptr(), 9280, torch.cuda.current_stream().cuda_stream)
        torch.cuda.current_stream().wait_stream(st)
        ref = sum(_data(r, 9280, 99) for r in range(world))
        for _ in range(4):
            g.replay()
            torch.cuda.synchronize()
            if (buf.cpu() - ref).abs().max().item() > 1e-5:
                errs.append("graph replay mismatch")
        if n.xar_status(x) != 0:
            errs.append("status reported a timeout in the healthy phase")
        dist.barrier()
        # bounded barrier: only rank 0 calls; it must time out, not hang
        if rank == 0:
            z = torch.ones(1024, device="cuda")
            n.xar_all_reduce_f32(x, z.data_ptr(), z.data_ptr(), 1024, s)
            torch.cuda.synchronize()
            if n.xar_status(x) != -1:
                errs.append("missing peer did not time out")
        dist.barrier()
        n.xar_destroy(x)
        dist.destroy_process_group()
        q.put((rank, errs))
    except Exception as e:  # noqa: BLE001
        q.put((rank, [repr(e)]))


@pytest.mark.gpu
@pytest.mark.parametrize("world,mode", [(2, "1"), (2, "2"), (3, "2"), (4, "0"), (8, "0"), (8, "1")])
def test_xgmi_allreduce_processes(gpu, world, mode):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=110) for _ in ps)
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert res == {r: [] for r in range(world)}, res
