"""The 256-sample tile front kernel (csrc/gpu/kernels_mlp3t.hip, mlp3_tile) against its
PyTorch emulation (ops.mlp3_tile on CPU tensors: the same rounding points, FP32 sums) and
the per-layer path, for every output type, label / dense targets, n_out <= 16 and > 16,
padded batches and several tiles per workgroup."""
import pytest
import torch

from hpnn_amd import ops
from hpnn_amd.models import MLP


def _case(net, n_out, Bp, u8, seed):
    torch.manual_seed(seed)
    m = MLP([784, 128, 64, n_out], net, batch=Bp, momentum=True, seed=seed, fused="t")
    if u8:
        X = torch.randint(0, 256, (Bp, 784), dtype=torch.uint8)
    else:
        X = torch.rand(Bp, 784) - 0.5
    return m, X


@pytest.mark.gpu
@pytest.mark.parametrize("net,n_out,dense,u8,Bp,n_valid,grid", [
    ("SNN", 10, False, True, 4096, 4096, 0),
    ("SNN", 10, False, False, 2048, 1999, 0),
    ("SNN", 24, True, True, 2048, 2048, 3),   # dense targets, 2 output tiles, 3 WGs x several tiles
    ("ANN", 10, True, False, 1024, 1000, 0),
    ("ANN", 30, False, True, 1024, 1024, 1),  # one WG runs every tile
    ("LNN", 12, True, False, 512, 512, 0),
])
def test_tile_kernel_matches_emulation(gpu, net, n_out, dense, u8, Bp, n_valid, grid):
    m, X = _case(net, n_out, Bp, u8, seed=Bp + n_out)
    Xg = m.prepare_input(X.cuda())
    t_hi, t_lo = (1.0, 0.0) if net == "SNN" else (1.0, -1.0)
    lab = torch.randint(0, n_out, (Bp,), dtype=torch.int32)
    T = None
    if dense:
        T = torch.full((Bp, n_out), t_lo)
        T[torch.arange(Bp), lab.long()] = t_hi
    G = grid or ops.mlp3_tile_grid(Bp)
    gslab = torch.zeros(G, ops.MLP3_SLAB, device="cuda")
    D1 = torch.zeros(Bp // 32, 8, 64, 8, dtype=torch.bfloat16, device="cuda")
    stats = torch.zeros(64, 16, device="cuda")
    ty = {"ANN": ops.TYPE_ANN, "LNN": ops.TYPE_LNN, "SNN": ops.TYPE_SNN}[net]
    kw = dict(T=T.cuda()) if dense else dict(labels=lab.cuda())
    ops.mlp3_tile(Xg, 800, m.Wb[0], m.W0f, m.Wb[1], m.Wb[2], m.Wt[2], D1, gslab, n_out, ty, t_hi=t_hi, t_lo=t_lo,
                  n_valid=n_valid, loss_acc=stats[0, 0:1], correct=stats[0, 1:2], xscale=Xg.hpnn_fm_scale, **kw)
    torch.cuda.synchronize()
    # emulation on the CPU copies of the same operands
    Xc = Xg.cpu()
    gs_ref = torch.zeros(1, ops.MLP3_SLAB)
    D1_ref = torch.zeros(Bp // 32, 8, 64, 8, dtype=torch.bfloat16)
    st_ref = torch.zeros(64, 16)
    kwc = dict(T=T) if dense else dict(labels=lab)
    ops.mlp3_tile(Xc, 800, m.Wb[0].cpu(), None, m.Wb[1].cpu(), m.Wb[2].cpu(), m.Wt[2].cpu(), D1_ref, gs_ref, n_out,
                  ty, t_hi=t_hi, t_lo=t_lo, n_valid=n_valid, loss_acc=st_ref[0, 0:1], correct=st_ref[0, 1:2],
                  xscale=Xg.hpnn_fm_scale, **kwc)
    d1 = ops.from_fragment_major(D1.cpu(), Bp, 128).float()
    d1r = ops.from_fragment_major(D1_ref, Bp, 128).float()
    # bf16 outputs: a 1-ulp flip of an intermediate is allowed, systematic error is not
    scale = d1r.abs().max().item() + 1e-6
    assert (d1 - d1r).abs().max().item() < 0.05 * scale
    assert (d1 - d1r).abs().mean().item() < 2e-3 * scale
    assert torch.count_nonzero(d1[n_valid:]) == 0
    g = gslab.sum(0).cpu()
    gr = gs_ref[0]
    assert (g - gr).abs().max().item() < 0.02 * (gr.abs().max().item() + 1e-6), (g - gr).abs().max()
    loss, hits = float(stats[:, 0].sum()), int(stats[:, 1].contiguous().view(torch.int32).sum())
    loss_r, hits_r = float(st_ref[0, 0]), int(st_ref[0, 1:2].view(torch.int32).item())
    assert abs(loss - loss_r) <= 2e-3 * abs(loss_r) + 1e-3, (loss, loss_r)
    assert abs(hits - hits_r) <= max(2, n_valid // 200), (hits, hits_r)


@pytest.mark.gpu
@pytest.mark.parametrize("u8", [True, False])
def test_tile_train_step_matches_layerwise(gpu, u8):
    """whole steps (front + G0 + update) on the tile path vs the per-layer kernels"""
    Bp, n_out = 8192, 10
    mt, X = _case("SNN", n_out, Bp, u8, seed=3)
    ml = MLP([784, 128, 64, n_out], "SNN", batch=Bp, momentum=True, seed=3, fused=False)
    Xt, Xl = mt.prepare_input(X.cuda()), ml.prepare_input(X.cuda())
    lab = torch.randint(0, n_out, (Bp,), dtype=torch.int32, device="cuda")
    for _ in range(3):
        mt.train_step(Xt, labels=lab, lr=0.05)
        ml.train_step(Xl, labels=lab, lr=0.05)
    torch.cuda.synchronize()
    for a, b in zip(mt.host_weights(), ml.host_weights()):
        assert (a - b).abs().max().item() < 2e-3 * (b.abs().max().item() + 1e-3)
    (la, ca), (lb, cb) = mt.read_stats(), ml.read_stats()
    assert abs(la - lb) <= 1e-2 * abs(lb) and abs(ca - cb) <= 0.01 * Bp
    # predictions through the fragment-major input agree with the row-major path
    assert (mt.predict(Xt) - ml.predict(Xl)).abs().max().item() < 0.05


@pytest.mark.gpu
def test_tile_bitwise_repeatable(gpu):
    Bp = 4096
    ms = []
    for _ in range(2):
        m, X = _case("SNN", 10, Bp, True, seed=11)
        Xg = m.prepare_input(X.cuda())
        lab = torch.randint(0, 10, (Bp,), dtype=torch.int32, device="cuda")
        for _ in range(2):
            m.train_step(Xg, labels=lab)
        ms.append(m)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(ms[0].W32, ms[1].W32))


@pytest.mark.gpu
@pytest.mark.parametrize("Bp", [24576, 4096])
def test_fused_g0_update_matches_separate_update(gpu, Bp):
    """G0 with its split-K reduction and every layer's step in one launch
    (kernels_g0.hip g0_fused_kernel: write-through partials, per-tile tickets, fixed-order
    reduction) == G0 slabs + the sgd_update_multi launch, up to the order of the FP32 sums;
    and bitwise repeatable run to run (24576: 48 splits, the headline's split count)"""
    runs = {}
    for tag, fused in (("fused", True), ("fused2", True), ("sep", False)):
        m, X = _case("SNN", 10, Bp, True, seed=5)
        m.plan.g0_fused = fused
        Xg = m.prepare_input(X.cuda())
        g = torch.Generator(device="cuda").manual_seed(9)
        W0 = [w.clone() for w in m.W32]
        for _ in range(3):
            lab = torch.randint(0, 10, (Bp,), dtype=torch.int32, device="cuda", generator=g)
            m.train_step(Xg, labels=lab, lr=0.05)
        torch.cuda.synchronize()
        assert m.plan.health(torch.cuda.current_stream().cuda_stream) == 0
        runs[tag] = (m, W0)
    a, b = runs["fused"][0], runs["sep"][0]
    for l in range(3):
        assert torch.equal(a.W32[l], runs["fused2"][0].W32[l])  # repeatable
        assert torch.equal(a.Wb[l], runs["fused2"][0].Wb[l]) and torch.equal(a.Wt[l], runs["fused2"][0].Wt[l])
        dw = (b.W32[l] - runs["sep"][1][l]).abs().max().item()
        assert (a.W32[l] - b.W32[l]).abs().max().item() <= 1e-4 * dw + 1e-7, l
        assert torch.equal(a.Wb[l], a.W32[l].bfloat16()) and torch.equal(a.Wt[l], a.W32[l].bfloat16().t())
        dv = (b.V32[l]).abs().max().item()
        assert (a.V32[l] - b.V32[l]).abs().max().item() <= 1e-4 * dv + 1e-8, l
    from hpnn_amd import ops
    assert torch.equal(a.W0f, ops.frag_major(a.W32[0].bfloat16()))


@pytest.mark.gpu
def test_fused_g0_gradient_out_matches_slab_sums(gpu):
    """data-parallel form of the fused G0 launch (hpnn_g0_update.gout): no step, the reduced
    G0 and [G1|G2] land in the plan's flat gradient buffer -> grads_slabs returns ONE segment
    (the xGMI exchange then moves one copy instead of summing 48 + groups slabs) equal to the
    sums of the unfused slab segments; bitwise repeatable"""
    Bp = 24576
    out = {}
    for tag, fused in (("fused", True), ("fused2", True), ("sep", False)):
        m, X = _case("SNN", 10, Bp, True, seed=5)
        m.plan.g0_fused = fused
        Xg = m.prepare_input(X.cuda())
        lab = torch.randint(0, 10, (Bp,), dtype=torch.int32, device="cuda",
                            generator=torch.Generator(device="cuda").manual_seed(9))
        segs = m.grads_slabs(Xg, labels=lab)
        torch.cuda.synchronize()
        if fused:
            assert len(segs) == 1 and segs[0][0] == m.grad_flat.data_ptr() and segs[0][2] == 1, segs
            out[tag] = m.grad_flat.clone()
        else:
            assert len(segs) == 2
            parts = []
            for addr, stride, cnt, n in segs:
                base = [t for t in (m.slab[0], m.midtmp) if t.data_ptr() == addr][0].view(-1)
                parts.append(torch.stack([base[s * stride:s * stride + n] for s in range(cnt)]).sum(0))
            out[tag] = torch.cat(parts)[:m.grad_flat.numel()]
        assert m.plan.health(torch.cuda.current_stream().cuda_stream) == 0
    assert torch.equal(out["fused"], out["fused2"])
    ref = out["sep"]
    assert ((out["fused"] - ref).abs().max() <= 1e-5 * ref.abs().max()).item()
