"""First-layer weight gradient over fragment-major operands (csrc/gpu/kernels_g0.hip) and
the fused front's fragment-major delta1 (kernels_mlp3x.hip, d1fm).

Numerics against a plain PyTorch fp32 reference of the same product; the fragment-major
delta1 against the row-major one of the same kernel; a training step on the
fragment-major path against the LDS-staged TN path (same math, other summation order)."""
import pytest
import torch

from hpnn_amd import ops
from hpnn_amd.models import MLP


def _bf(*shape, scale=1.0):
    return ((torch.rand(*shape, device="cuda") - 0.5) * scale).bfloat16()


@pytest.mark.gpu
@pytest.mark.parametrize("Bt,N,M,S", [(65536, 128, 800, 48), (65536, 128, 800, 51), (4096, 128, 800, 5),
                                      (2048, 64, 64, 7), (1024, 32, 96, 3), (8192, 128, 832, 16),
                                      (8192, 128, 832, 12)])
def test_gemm_fm_direct_matches_fp32(gpu, Bt, N, M, S):
    torch.manual_seed(Bt + N + M)
    D, H = _bf(Bt, N, scale=0.25), _bf(Bt, M)
    slab = ops.gemm_fm_direct(ops.to_fragment_major(D), ops.to_fragment_major(H), N, M, splits=S)
    torch.cuda.synchronize()
    ref = D.float().t() @ H.float()
    got = slab.sum(0)
    err = (got - ref).abs().max().item()
    assert err < 1e-5 * Bt ** 0.5 * 4 + 1e-4, err
    # per-split slabs: split s covers batch rows [s*U/S, (s+1)*U/S) of 32-row units (every
    # split: the XCD-aware block order maps 8 * (S // 8) of them by XCD, the rest in order)
    U = Bt // 32
    for s in range(S):
        a, b = 32 * (s * U // S), 32 * ((s + 1) * U // S)
        ref_s = D[a:b].float().t() @ H[a:b].float()
        assert (slab[s] - ref_s).abs().max().item() < 1e-3, s


@pytest.mark.gpu
def test_gemm_fm_direct_with_tail_reduce(gpu):
    torch.manual_seed(5)
    Bt, N, M, S = 16384, 128, 800, 16
    D, H = _bf(Bt, N, scale=0.25), _bf(Bt, M)
    rslab = torch.randn(40, ops.MLP3_SLAB, device="cuda")
    groups = 8
    rout = torch.empty(groups, ops.MLP3_SLAB, device="cuda")
    slab = torch.empty(S, N, M, device="cuda")
    ops.gemm_fm_direct_reduce(ops.to_fragment_major(D), ops.to_fragment_major(H), N, M, S, slab, rslab, groups, rout)
    torch.cuda.synchronize()
    assert (slab.sum(0) - D.float().t() @ H.float()).abs().max().item() < 2e-3
    SG = (40 + groups - 1) // groups
    for g in range(groups):
        ref = rslab[g * SG:min(40, (g + 1) * SG)].sum(0)
        assert (rout[g] - ref).abs().max().item() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("net", ["SNN", "ANN"])
def test_fused_front_fragment_major_delta1(gpu, net):
    torch.manual_seed(7)
    B = 8192
    m = MLP([784, 128, 64, 10], net, batch=B, seed=2, fused="x")
    X = m.prepare_input(torch.rand(B, 784))
    X.hpnn_fm = ops.to_fragment_major(X)  # a fragment-major copy attached by hand
    assert m._fm_input(X) is not None
    lab = torch.randint(0, 10, (B,), dtype=torch.int32, device="cuda")
    Xrm = X.clone()  # no fragment-major copy attached: row-major delta1
    assert m._fm_input(Xrm) is None
    m._fused_front(Xrm, lab, None, B - 3)
    d_rm = m.D[0].clone()
    s_rm = m.midslab.clone()
    m._fused_front(X, lab, None, B - 3)
    d_fm = ops.from_fragment_major(m.D[0].view(-1), B, 128)
    torch.cuda.synchronize()
    diff = (d_fm.float() - d_rm.float()).abs()
    # same products, operands swapped in the MFMA: at most one bf16 rounding step apart
    assert diff.max().item() <= 2 ** -7 * d_rm.float().abs().max().item() + 1e-6
    assert (diff > 0).float().mean().item() < 0.01
    assert torch.equal(m.midslab, s_rm)


@pytest.mark.gpu
def test_train_step_fragment_major_matches_tn(gpu):
    torch.manual_seed(9)
    B = 16384
    ms = [MLP([784, 128, 64, 10], "SNN", batch=B, seed=3, momentum=True, fused="x") for _ in range(2)]
    xs = [torch.rand(B, 784) for _ in range(3)]
    labs = [torch.randint(0, 10, (B,), dtype=torch.int32, device="cuda") for _ in range(3)]
    for i, m in enumerate(ms):
        for x, lab in zip(xs, labs):
            X = m.prepare_input(x)
            if i == 0:
                X.hpnn_fm = ops.to_fragment_major(X)  # fragment-major G0 path (copy attached by hand)
            m.train_step(X, labels=lab, lr=0.05, alpha=0.2)
    torch.cuda.synchronize()
    for l in range(3):
        e = (ms[0].W32[l] - ms[1].W32[l]).abs().max().item()
        assert e < 1e-5, (l, e)


@pytest.mark.gpu
def test_gemm_fm_direct_u8_pixels(gpu):
    """8-bit operand: the kernel multiplies the exact integers (BF16 holds 0..255 exactly)
    and applies hscale to the FP32 accumulator, so it matches D^T (pixels * hscale) in FP32,
    not the BF16-rounded pixels / 255"""
    torch.manual_seed(21)
    Bt, N, M, S = 16384, 128, 800, 16
    D = _bf(Bt, N, scale=0.25)
    Hu = torch.randint(0, 256, (Bt, M), device="cuda", dtype=torch.uint8)
    sc = float(torch.tensor(1.0 / 255.0, dtype=torch.float32).item())
    slab = ops.gemm_fm_direct(ops.to_fragment_major(D), ops.to_fragment_major(Hu), N, M, splits=S, hscale=sc)
    ref_int = ops.gemm_fm_direct(ops.to_fragment_major(D), ops.to_fragment_major(Hu.bfloat16()), N, M, splits=S)
    torch.cuda.synchronize()
    ref = (D.float().t() @ Hu.float()) * sc
    assert (slab.sum(0) - ref).abs().max().item() < 1e-4 * ref.abs().max().item()
    # the same integer products as the BF16 kernel on the integers, scaled once per slab
    assert (slab - ref_int * sc).abs().max().item() < 1e-5 * ref_int.abs().max().item() * sc


@pytest.mark.gpu
@pytest.mark.parametrize("fused", ["x", "t"])
def test_train_step_u8_pixels_matches_float(gpu, fused):
    """uint8 pixel input (exact integers, the pixel scale on the FP32 accumulators) vs the
    same pixels given as floats pixel/255 (rounded to BF16 once at input preparation).  The
    operands differ by BF16 input rounding (|rel| <= 2^-9 per pixel, unbiased), so after 3
    steps the weights agree to the accumulated rounding, not bitwise: measured up to 2.2e-3
    of a layer's largest weight change (layer 1, tile path; the differing inputs flip BF16
    roundings of H1 downstream), gated at 5e-3."""
    torch.manual_seed(23)
    B = 16384
    ms = [MLP([784, 128, 64, 10], "SNN", batch=B, seed=3, momentum=True, fused=fused) for _ in range(2)]
    W0 = [w.clone() for w in ms[0].W32]
    from hpnn_amd.models.mlp import PIXEL_SCALE
    for step in range(3):
        xu = torch.randint(0, 256, (B, 784), dtype=torch.uint8)
        lab = torch.randint(0, 10, (B,), dtype=torch.int32, device="cuda")
        Xa = ms[0].prepare_input(xu)
        Xb = ms[1].prepare_input(xu.float() * PIXEL_SCALE)
        if fused == "x":
            assert ms[0]._fm_input(Xa) is not None and ms[0]._fm_input(Xa).dtype == torch.uint8
            assert ms[1]._fm_input(Xb) is None
        else:
            assert Xa.dtype == torch.uint8 and Xb.dtype == torch.bfloat16
        ms[0].train_step(Xa, labels=lab, lr=0.05, alpha=0.2)
        ms[1].train_step(Xb, labels=lab, lr=0.05, alpha=0.2)
    torch.cuda.synchronize()
    for l in range(3):
        da, db = ms[0].W32[l] - W0[l], ms[1].W32[l] - W0[l]
        e = (da - db).abs().max().item()
        assert e < 5e-3 * db.abs().max().item(), (l, e, db.abs().max().item())
