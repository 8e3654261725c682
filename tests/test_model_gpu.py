"""End-to-end batched training step on the GPU vs the FP64 PyTorch oracle."""
import pytest
import torch

from hpnn_amd import ops

from hpnn_amd.models import MLP
from hpnn_amd.models import reference as ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("net_type,sizes,momentum", [
    ("SNN", [784, 128, 64, 10], True),
    ("SNN", [784, 128, 64, 10], False),
    ("ANN", [64, 96, 32], False),
    ("LNN", [40, 64, 8], True),
    ("SNN", [300, 230, 230], True),
    ("SNN", [4096, 230, 230], True),     # RRUFF shape: the wide-input front ("w")
    ("ANN", [4096, 4096, 4096], True),   # full-width 4096 x 4096 layer pair (8-phase GEMMs)
])
def test_train_step_matches_oracle(gpu, net_type, sizes, momentum):
    """3 steps vs FP64 math on the same BF16-rounded inputs and initial weights.  The
    kernels round activations and deltas to BF16 (8 significant bits, 2^-9 relative per
    rounding) and the weights to BF16 for every GEMM, with FP32 accumulation; measured
    relative error of the weight change (Frobenius): 2e-3 .. 6e-3 over these nets, loss
    sum within 3e-3 -- the bounds below leave ~2x headroom."""
    torch.manual_seed(0)
    B = 256
    # reference_init (the reference's serial random() stream) is for small nets; the
    # 4096 x 4096 pair takes the fast seeded rule (the oracle starts from m's own weights)
    init = "fast" if max(a * b for a, b in zip(sizes, sizes[1:])) > 4_000_000 else "reference"
    m = MLP(sizes, net_type, batch=B, momentum=momentum, seed=7, init=init)
    W64 = [w.clone() for w in m.host_weights()]
    V64 = [torch.zeros_like(w) for w in W64] if momentum else None
    X = torch.rand(B, sizes[0], dtype=torch.float64)
    labels = torch.randint(0, sizes[-1], (B,))
    lo = 0.0 if net_type == "SNN" else -1.0
    T = torch.full((B, sizes[-1]), lo, dtype=torch.float64)
    T[torch.arange(B), labels] = 1.0
    # the oracle sees the same bf16-rounded inputs and weights the kernels see
    Xb = X.float().bfloat16().double()
    Xd = m.prepare_input(X)
    lab = labels.to(torch.int32).cuda()
    loss_total = 0.0
    for step in range(3):
        m.train_step(Xd, labels=lab, lr=0.05, alpha=0.2)
        loss_total += ref.batched_step(W64, Xb, T, net_type, 0.05, V64, 0.2).item()
    torch.cuda.synchronize()
    got = m.host_weights()
    W0 = [w.float().double() for w in MLP(sizes, net_type, batch=B, momentum=momentum, seed=7, init=init).host_weights()]
    for l in range(len(got)):
        dg = got[l] - W0[l]
        dr = W64[l] - W0[l]
        rel = (dg - dr).norm() / (dr.norm() + 1e-30)
        print(f"{net_type} {sizes} layer {l}: relative error of the weight change {rel.item():.2e}")
        assert rel < 0.012, (l, rel.item())
    lsum, corr = m.read_stats()
    print(f"loss sum {lsum:.6g} vs oracle {loss_total * B:.6g}")
    assert lsum == pytest.approx(loss_total * B, rel=6e-3)


def test_predict_matches_forward(gpu):
    m = MLP([784, 128, 64, 10], "SNN", batch=128, seed=3)
    X = torch.rand(100, 784, dtype=torch.float64)
    O = m.predict(m.prepare_input(X), n_valid=100).cpu().double()
    R = ref.forward([w.float().bfloat16().double() for w in m.host_weights()], X.float().bfloat16().double(), "SNN")[-1]
    assert (O - R).abs().max().item() < 2e-2
    assert torch.allclose(O.sum(1), torch.ones(100, dtype=torch.float64), atol=1e-4)


@pytest.mark.parametrize("net_type", ["SNN", "ANN", "LNN"])
@pytest.mark.parametrize("B,n_valid", [(1024, 1024), (640, 600), (16384, 16000), (40960, 40000)])
@pytest.mark.parametrize("mode,n_in", [("x", 784), ("mid", 784), ("x", 250)])
def test_fused_matches_layerwise(gpu, net_type, B, n_valid, mode, n_in):
    """fused mlp3 paths == per-layer path (same math, different summation order)."""
    torch.manual_seed(1)
    sizes = [n_in, 128, 64, 10]
    mf = MLP(sizes, net_type, batch=B, momentum=True, seed=5, fused=mode, mid_grid=3)
    assert mf.fused_mode == mode
    ml = MLP(sizes, net_type, batch=B, momentum=True, seed=5, fused=False)
    assert mf.fused and not ml.fused
    X = torch.rand(mf.Bp, n_in)
    labels = torch.randint(0, 10, (mf.Bp,), dtype=torch.int32).cuda()
    Xd = mf.prepare_input(X)
    for _ in range(2):
        mf.train_step(Xd, labels=labels, n_valid=n_valid, lr=0.05)
        ml.train_step(Xd, labels=labels, n_valid=n_valid, lr=0.05)
    torch.cuda.synchronize()
    for a, b in zip(mf.host_weights(), ml.host_weights()):
        assert (a - b).abs().max().item() < 2e-3 * (b.abs().max().item() + 1e-3)
    la, ca = mf.read_stats()
    lb, cb = ml.read_stats()
    assert la == pytest.approx(lb, rel=2e-2)
    assert abs(ca - cb) <= max(2, 0.01 * n_valid)
    D1 = mf.D[0]
    if mf._fm_input(Xd) is not None:  # delta1 fragment-major (first-layer gradient kernel operand)
        D1 = ops.from_fragment_major(D1.view(-1), mf.Bp, 128)
    assert torch.equal(D1[n_valid:], torch.zeros_like(D1[n_valid:]))


@pytest.mark.parametrize("net_type", ["SNN", "ANN"])
def test_fused_x_dense_targets(gpu, net_type):
    """mlp3_fused with dense targets T (no labels) == the per-layer path with T."""
    torch.manual_seed(2)
    sizes, B = [784, 128, 64, 20], 2048
    mf = MLP(sizes, net_type, batch=B, momentum=False, seed=9, fused="x")
    ml = MLP(sizes, net_type, batch=B, momentum=False, seed=9, fused=False)
    X = mf.prepare_input(torch.rand(B, 784))
    lo = 0.0 if net_type == "SNN" else -1.0
    T = torch.full((B, 20), lo, device="cuda")
    T[torch.arange(B), torch.randint(0, 20, (B,))] = 1.0
    for m in (mf, ml):
        m.train_step(X, T=T, lr=0.05)
    torch.cuda.synchronize()
    for a, b in zip(mf.host_weights(), ml.host_weights()):
        assert (a - b).abs().max().item() < 2e-3 * (b.abs().max().item() + 1e-3)
    assert mf.read_stats()[0] == pytest.approx(ml.read_stats()[0], rel=2e-2)
    assert abs(mf.read_stats()[1] - ml.read_stats()[1]) <= 20


def test_fused_x_kernel_vs_emulation(gpu):
    """kernel outputs (delta1, [G1|G2] slab sum, loss, hits) vs the PyTorch emulation
    with the same rounding points; W0f is the fragment-major copy the update writes."""
    from hpnn_amd import ops
    torch.manual_seed(3)
    sizes, B = [784, 128, 64, 10], 8192
    m = MLP(sizes, "SNN", batch=B, seed=4, fused="x")
    assert torch.equal(m.W0f, ops.frag_major(m.Wb[0]))
    X = m.prepare_input(torch.rand(B, 784))
    lab = torch.randint(0, 10, (B,), dtype=torch.int32, device="cuda")
    m.reset_stats()
    m._fused_front(X, lab, None, B - 5)
    torch.cuda.synchronize()
    slab = torch.zeros(1, ops.MLP3_SLAB)
    D1 = torch.empty(B, 128, dtype=torch.bfloat16)
    st = torch.zeros(64, 16)
    ops.mlp3_fused(X.cpu(), m.Wb[0].cpu(), None, m.Wb[1].cpu(), m.Wb[2].cpu(), D1, slab, 10, ops.TYPE_SNN,
                   labels=lab.cpu(), n_valid=B - 5, loss_acc=st[0, 0:1], correct=st[0, 1:2])
    got_d1 = m.D[0].cpu()
    if m._fm_input(X) is not None:  # delta1 was written fragment-major for the G0 kernel
        got_d1 = ops.from_fragment_major(got_d1.view(-1), B, 128)
    d = (got_d1.float() - D1.float()).abs().max().item()
    assert d < 2e-2 * (D1.float().abs().max().item() + 1e-6), d
    got = m.midslab.sum(0).cpu()
    ref_ = slab[0]
    assert (got - ref_).abs().max().item() < 2e-2 * (ref_.abs().max().item() + 1e-6)
    loss, hits = m.read_stats()
    assert loss == pytest.approx(st[0, 0].item(), rel=1e-2)
    assert abs(hits - ops_hits(st)) <= 40


def ops_hits(st):
    return int(st[:, 1].contiguous().view(torch.int32).long().sum())


def test_update_multi_writes_fragment_major(gpu):
    from hpnn_amd import ops
    torch.manual_seed(5)
    W = torch.randn(128, 800, device="cuda")
    V = torch.zeros_like(W)
    G = torch.randn(4, 128, 800, device="cuda")
    Wb = torch.empty(128, 800, dtype=torch.bfloat16, device="cuda")
    Wt = torch.empty(800, 128, dtype=torch.bfloat16, device="cuda")
    Wf = torch.empty(128 * 800, dtype=torch.bfloat16, device="cuda")
    W2 = torch.randn(64, 128, device="cuda")
    G2 = torch.randn(128 * 64 * 3, device="cuda")[:64 * 128 * 3].view(3, 64, 128)
    W2b = torch.empty(64, 128, dtype=torch.bfloat16, device="cuda")
    W2t = torch.empty(128, 64, dtype=torch.bfloat16, device="cuda")
    Wr, W2r = W.clone(), W2.clone()
    ops.sgd_update_multi([(W, V, G, Wb, Wt, Wf), (W2, None, G2, W2b, W2t, None)], 0.1, 0.0, 0.5, False)
    torch.cuda.synchronize()
    assert torch.allclose(W, Wr + 0.1 * 0.5 * G.sum(0), atol=1e-5)
    assert torch.allclose(W2, W2r + 0.1 * 0.5 * G2.sum(0), atol=1e-5)
    assert torch.equal(Wb, W.bfloat16()) and torch.equal(Wt, W.bfloat16().t())
    assert torch.equal(Wf, ops.frag_major(Wb))
    assert torch.equal(W2t, W2.bfloat16().t())


@pytest.mark.parametrize("momentum", [True, False])
def test_tn_update_fused_matches_separate(gpu, momentum):
    """the weight gradient with the optimizer step in the 8-phase TN epilogue
    (ops.gemm_tn_update, one split, 256x256 tiles) against the separate gradient + update
    kernels: same weights / momentum to GEMM summation order, and the BF16 copies W / W^T
    written by the epilogue are the FP32 master rounded"""
    torch.manual_seed(3)
    sizes, B = [512, 512, 256], 2048
    ms = []
    for fused in (True, False):
        m = MLP(sizes, "ANN", batch=B, momentum=momentum, seed=11, init="fast", splits=[1, 1])
        m.tn_update = fused
        ms.append(m)
    assert all(ms[0]._tn_update_ok(l) for l in range(2)) and not ms[1]._tn_update_ok(0)
    X = torch.rand(B, sizes[0])
    T = torch.rand(B, sizes[-1], device="cuda") * 2 - 1
    for m in ms:
        Xd = m.prepare_input(X)
        for _ in range(3):
            m.train_step(Xd, T=T, lr=0.05, alpha=0.2)
    torch.cuda.synchronize()
    a, b = ms
    for l in range(2):
        W0 = b.W32[l]
        assert (a.W32[l] - W0).abs().max().item() <= 1e-5 * max(1.0, W0.abs().max().item())
        if momentum:
            assert (a.V32[l] - b.V32[l]).abs().max().item() <= 1e-5 * max(1e-3, b.V32[l].abs().max().item())
        assert torch.equal(a.Wb[l], a.W32[l].bfloat16())
        assert torch.equal(a.Wt[l], a.W32[l].bfloat16().t().contiguous())


@pytest.mark.parametrize("momentum", [True, False])
def test_production_step_matches_oracle(gpu, momentum):
    """The headline step itself (bench.py's config) against the FP64 oracle: MNIST
    784-128-64-10 SNN, batch 65 536, 8-bit pixels, the tile front + the fused first-layer
    gradient launch at its default split count (48: split-K reduction, optimizer steps and
    the [G1 | G2] share in one launch).  Two steps; the oracle runs in FP64 on the GPU on the
    same inputs (pixel / 255 rounded to BF16, as the front sees them) and the same initial
    weights.  Same bounds as test_train_step_matches_oracle.  Reference step math:
    snn.c:798-1074, batched."""
    torch.manual_seed(0)
    sizes, B, lr = [784, 128, 64, 10], 65536, 0.01
    m = MLP(sizes, "SNN", batch=B, momentum=momentum, seed=10958)
    assert m.fused_mode == "t"
    import ctypes
    from hpnn_amd._lib import lib_path
    ok = ctypes.CDLL(lib_path()).hpnn_gemm_fm_direct_update_ok
    assert m.plan.g0_fused and ok(m.Kp[0], m.Np[0], m.Kp[0], m.Bp, m.S[0]) == 1, "the fused G0 launch must run"
    g = torch.Generator(device="cuda").manual_seed(1234)
    Xu8 = torch.randint(0, 256, (B, 784), device="cuda", generator=g, dtype=torch.uint8)
    labels = torch.randint(0, 10, (B,), device="cuda", generator=g, dtype=torch.int32)
    Xd = m.prepare_input(Xu8)
    W64 = [w.cuda() for w in m.host_weights()]
    V64 = [torch.zeros_like(w) for w in W64] if momentum else None
    W0 = [w.clone() for w in W64]
    Xb = (Xu8.double() / 255.0).float().bfloat16().double()
    T = torch.zeros(B, 10, dtype=torch.float64, device="cuda")
    T[torch.arange(B, device="cuda"), labels.long()] = 1.0
    loss_total = 0.0
    m.reset_stats()
    for _ in range(2):
        m.train_step(Xd, labels=labels, lr=lr, alpha=0.2)
        loss_total += ref.batched_step(W64, Xb, T, "SNN", lr, V64, 0.2).item()
    torch.cuda.synchronize()
    assert m.healthy()
    got = [w.cuda() for w in m.host_weights()]
    for l in range(3):
        dg, dr = got[l] - W0[l], W64[l] - W0[l]
        rel = (dg - dr).norm() / (dr.norm() + 1e-30)
        print(f"production step layer {l}: relative error of the weight change {rel.item():.2e}")
        assert rel < 0.012, (l, rel.item())
    lsum, _ = m.read_stats()
    print(f"loss sum {lsum:.8g} vs oracle {loss_total * B:.8g}")
    assert lsum == pytest.approx(loss_total * B, rel=6e-3)
