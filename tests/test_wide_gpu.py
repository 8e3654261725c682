"""The wide-input front (csrc/gpu/kernels_wide.hip, ops.wide2_front) on the GPU:
  - against its PyTorch emulation (the same BF16 rounding points) for every output type,
    label / dense targets, padded batches and both work splits (1 or 2 workgroups per
    128-sample tile, the second handing its FP32 partial over through memory);
  - bitwise repeatable with the hand-over (a + b == b + a whichever workgroup finishes
    first);
  - one whole training step of the RRUFF-shaped 4096-230-230 SNN (mode "w") against an
    FP64 oracle of the same step (reference math: snn.c / ann.c back-propagation with
    momentum), and against the per-layer path."""
import pytest
import torch

from hpnn_amd import ops
from hpnn_amd.models import MLP

pytestmark = pytest.mark.gpu
TYPES = {"ANN": ops.TYPE_ANN, "LNN": ops.TYPE_LNN, "SNN": ops.TYPE_SNN}


def _front(net, n_out, dense, Bp, n_valid, ksplit, seed):
    torch.manual_seed(seed)
    m = MLP([4096, 230, n_out], net, batch=Bp, momentum=True, seed=seed, fused="w")
    X = m.prepare_input((torch.rand(Bp, 4096) - 0.3).cuda())
    t_hi, t_lo = (1.0, 0.0) if net == "SNN" else (1.0, -1.0)
    lab = torch.randint(0, n_out, (Bp,), dtype=torch.int32)
    kw = {"labels": lab}
    if dense:
        T = torch.full((Bp, n_out), t_lo)
        T[torch.arange(Bp), lab.long()] = t_hi
        kw = {"T": T}
    ws = ops.Wide2Workspace(Bp, 4096, "cuda", ksplit=ksplit)
    outs = [torch.zeros(Bp, 256, dtype=torch.bfloat16, device="cuda") for _ in range(3)]
    stats = torch.zeros(64, 16, device="cuda")
    ops.wide2_front(X, m.Wb[0], m.Wb[1], m.Wt[1], *outs, ws, n_out, TYPES[net], t_hi=t_hi, t_lo=t_lo,
                    n_valid=n_valid, loss_acc=stats[0, 0:1], correct=stats[0, 1:2],
                    **{k: v.cuda() for k, v in kw.items()})
    torch.cuda.synchronize()
    ws.check()
    ref = [torch.zeros(Bp, 256, dtype=torch.bfloat16) for _ in range(3)]
    st_ref = torch.zeros(64, 16)
    ops.wide2_front(X.cpu(), m.Wb[0].cpu(), m.Wb[1].cpu(), m.Wt[1].cpu(), *ref, None, n_out, TYPES[net], t_hi=t_hi,
                    t_lo=t_lo, n_valid=n_valid, loss_acc=st_ref[0, 0:1], correct=st_ref[0, 1:2], **kw)
    return [o.cpu() for o in outs], ref, stats.cpu(), st_ref, ws


@pytest.mark.parametrize("net,n_out,dense,Bp,n_valid,ksplit", [
    ("SNN", 230, False, 16384, 16384, 2),
    ("SNN", 230, False, 1024, 1000, 1),
    ("SNN", 256, True, 2048, 2048, 2),
    ("ANN", 230, True, 1024, 1000, 2),
    ("ANN", 240, False, 512, 512, 1),
    ("LNN", 230, False, 1024, 1024, 2),
])
def test_wide_front_matches_emulation(gpu, net, n_out, dense, Bp, n_valid, ksplit):
    outs, ref, st, st_ref, _ = _front(net, n_out, dense, Bp, n_valid, ksplit, seed=Bp + n_out)
    for name, a, b in zip(("H0", "delta2", "delta1"), outs, ref):
        a, b = a.float(), b.float()
        scale = b.abs().max().item() + 1e-6
        # BF16 outputs: a 1-ulp flip of an intermediate is allowed, systematic error is not
        assert (a - b).abs().max().item() < 0.05 * scale, name
        assert (a - b).abs().mean().item() < 2e-3 * scale, name
        assert torch.count_nonzero(a[n_valid:]) == 0 or name == "H0", name
    loss, hits = float(st[:, 0].sum()), int(st[:, 1].contiguous().view(torch.int32).sum())
    loss_r, hits_r = float(st_ref[0, 0]), int(st_ref[0, 1:2].view(torch.int32).item())
    assert abs(loss - loss_r) <= 2e-3 * abs(loss_r) + 1e-3, (loss, loss_r)
    assert abs(hits - hits_r) <= max(2, n_valid // 200), (hits, hits_r)


def test_wide_front_bitwise_repeatable_with_handover(gpu):
    a, _, sa, _, ws = _front("SNN", 230, False, 8192, 8192, 2, seed=5)
    b, _, sb, _, _ = _front("SNN", 230, False, 8192, 8192, 2, seed=5)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    assert torch.equal(sa[:, 1], sb[:, 1])
    # one launch: two tickets per tile on the monotonic counters, no exchange timed out
    n_tiles = 8192 // ops.WIDE2_TILE
    assert torch.equal(ws.cnt.cpu(), torch.full((n_tiles,), 2, dtype=torch.int32))
    assert int(ws.err.item()) == 0


def _oracle_step(W, V, X, lab, n_out, lr, alpha):
    """one momentum step of the 1-hidden-layer SNN in FP64 (unpadded weights)"""
    W0, W1 = W
    H = ops.bipolar(X @ W0.t())
    Z = H @ W1.t()
    T = torch.zeros(X.shape[0], n_out, dtype=torch.float64)
    T[torch.arange(X.shape[0]), lab.long()] = 1.0
    m = Z.max(1, keepdim=True).values
    e = torch.exp(Z - m)
    o = e / (e.sum(1, keepdim=True) + torch.exp(torch.log(torch.tensor(1e-14, dtype=torch.float64)) + 1.0 - m))
    d2 = T - o
    d1 = (d2 @ W1) * ops.dbipolar(H)
    G = [d1.t() @ X, d2.t() @ H]
    out = []
    for w, v, g in zip(W, V, G):
        v = v + lr * g / X.shape[0]
        out.append((w + v, v * alpha))
    return out


def test_rruff_step_against_fp64_oracle(gpu):
    """the whole 4096-230-230 step (wide front + weight gradients + momentum updates) vs
    FP64 math on the same BF16-representable inputs.  Measured error of the weight change
    (BF16 operands and activations, FP32 accumulation): see the bound's comment."""
    B, sizes, lr, alpha = 4096, [4096, 230, 230], 0.01, 0.2
    torch.manual_seed(1)
    m = MLP(sizes, "SNN", batch=B, momentum=True, seed=21)
    assert m.fused_mode == "w"
    X = torch.rand(B, sizes[0]).bfloat16().float()
    lab = torch.randint(0, sizes[-1], (B,), dtype=torch.int32)
    W_before = [w.double() for w in m.host_weights()]
    # the BF16 weights the kernels use (the FP32 masters are not BF16-representable)
    Wb = [m.Wb[l][:sizes[l + 1], :sizes[l]].double().cpu() for l in range(2)]
    m.train_step(m.prepare_input(X.cuda()), labels=lab.cuda(), lr=lr, alpha=alpha)
    torch.cuda.synchronize()
    dW = [a - b for a, b in zip(m.host_weights(), W_before)]
    ref = _oracle_step(Wb, [torch.zeros_like(w) for w in Wb], X.double(), lab, sizes[-1], lr, alpha)
    for l in range(2):
        dref = ref[l][0] - Wb[l]
        rel = ((dW[l] - dref).norm() / dref.norm()).item()
        mx = ((dW[l] - dref).abs().max() / dref.abs().max()).item()
        print(f"layer {l}: relative Frobenius error of the weight change {rel:.3e}, max-norm {mx:.3e}")
        # BF16 activations / deltas (8 significant bits, ~0.4% per rounding, several
        # roundings in a chain, errors averaging over the 4096-sample sums)
        assert rel < 2e-2 and mx < 5e-2, (l, rel, mx)


def test_rruff_step_wide_vs_layerwise(gpu):
    B, sizes = 16384, [4096, 230, 230]
    torch.manual_seed(2)
    mw = MLP(sizes, "SNN", batch=B, momentum=True, seed=3)
    ml = MLP(sizes, "SNN", batch=B, momentum=True, seed=3, fused=False)
    assert mw.fused_mode == "w" and ml.fused_mode is None
    X = torch.rand(B, sizes[0]).cuda()
    lab = torch.randint(0, sizes[-1], (B,), dtype=torch.int32, device="cuda")
    Xw, Xl = mw.prepare_input(X), ml.prepare_input(X)
    for _ in range(3):
        mw.train_step(Xw, labels=lab, lr=0.01, alpha=0.2)
        ml.train_step(Xl, labels=lab, lr=0.01, alpha=0.2)
    torch.cuda.synchronize()
    assert mw.plan.health(torch.cuda.current_stream().cuda_stream) == 0
    for a, b in zip(mw.host_weights(), ml.host_weights()):
        assert (a - b).abs().max().item() < 2e-3 * (b.abs().max().item() + 1e-3)
    (la, ca), (lb, cb) = mw.read_stats(), ml.read_stats()
    assert abs(la - lb) <= 1e-3 * abs(lb) and abs(ca - cb) <= 0.002 * 3 * B


@pytest.mark.parametrize("B", [8192])
def test_rruff_fused_tn8_update_matches_separate_update(gpu, B):
    """the RRUFF-shaped first layer's gradient over 16 split-K slices reduced and stepped
    inside the 8-phase TN launch (kernels_8ph.hip MODE 2: write-through partials, per-tile
    tickets, fixed-order sums) == slabs + the separate update launch, up to the order of the
    FP32 sums; bitwise repeatable run to run"""
    sizes = [4096, 230, 230]
    runs = {}
    for tag, fused in (("fused", True), ("fused2", True), ("sep", False)):
        torch.manual_seed(4)
        m = MLP(sizes, "SNN", batch=B, momentum=True, seed=8)
        assert m.fused_mode == "w" and m.S[0] > 1
        m.plan.g0_fused = fused
        X = m.prepare_input(torch.rand(B, sizes[0]).cuda())
        W0 = [w.clone() for w in m.W32]
        for i in range(3):
            lab = torch.randint(0, sizes[-1], (B,), dtype=torch.int32, device="cuda")
            m.train_step(X, labels=lab, lr=0.01, alpha=0.2)
        torch.cuda.synchronize()
        assert m.plan.health(torch.cuda.current_stream().cuda_stream) == 0
        runs[tag] = (m, W0)
    a, b = runs["fused"][0], runs["sep"][0]
    for l in range(2):
        assert torch.equal(a.W32[l], runs["fused2"][0].W32[l]) and torch.equal(a.Wt[l], runs["fused2"][0].Wt[l])
        dw = (b.W32[l] - runs["sep"][1][l]).abs().max().item()
        assert (a.W32[l] - b.W32[l]).abs().max().item() <= 1e-4 * dw + 1e-7, l
        assert torch.equal(a.Wb[l], a.W32[l].bfloat16()) and torch.equal(a.Wt[l], a.W32[l].bfloat16().t())


@pytest.mark.parametrize("B,momentum", [(16384, True), (8192, False)])
def test_rruff_layer1_side_job_bitwise(gpu, B, momentum):
    """layer 1's gradient + step carried by layer 0's fused TN launch as its side job
    (kernels_8ph.hip side_jobs / side_reduce_step) == the separate gemm_tn + update launches,
    BITWISE: the same 64 x 64 split-K pieces, the slab sum in sgd_tile's order.  Checks that the
    side path ran (plan.side_launches) and that the separate run did not take it."""
    sizes = [4096, 230, 230]
    runs = {}
    for tag, side in (("side", True), ("sep", False)):
        torch.manual_seed(5)
        m = MLP(sizes, "SNN", batch=B, momentum=momentum, seed=9)
        assert m.fused_mode == "w"
        m.plan.tn8_side = side
        X = m.prepare_input(torch.rand(B, sizes[0]).cuda())
        for _ in range(3):
            lab = torch.randint(0, sizes[-1], (B,), dtype=torch.int32, device="cuda")
            m.train_step(X, labels=lab, lr=0.01, alpha=0.2)
        torch.cuda.synchronize()
        assert m.plan.health(torch.cuda.current_stream().cuda_stream) == 0
        runs[tag] = m
    a, b = runs["side"], runs["sep"]
    assert b.plan.side_launches == 0
    if a.plan.side_launches == 0:
        pytest.skip(f"side job does not fit this grid (B={B}, splits {list(a.S)})")
    assert a.plan.side_launches == 3
    for l in range(2):
        assert torch.equal(a.W32[l], b.W32[l]), l
        if momentum:
            assert torch.equal(a.V32[l], b.V32[l]), l
        assert torch.equal(a.Wb[l], b.Wb[l]) and torch.equal(a.Wt[l], b.Wt[l]), l
        assert torch.equal(a.Wt[l], a.W32[l].bfloat16().t()), l
