"""End-to-end batched training step on the GPU vs the FP64 PyTorch oracle."""
import pytest
import torch

from hpnn_amd.models import MLP
from hpnn_amd.models import reference as ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("net_type,sizes,momentum", [
    ("SNN", [784, 128, 64, 10], True),
    ("SNN", [784, 128, 64, 10], False),
    ("ANN", [64, 96, 32], False),
    ("LNN", [40, 64, 8], True),
    ("SNN", [300, 230, 230], True),
])
def test_train_step_matches_oracle(gpu, net_type, sizes, momentum):
    torch.manual_seed(0)
    B = 256
    m = MLP(sizes, net_type, batch=B, momentum=momentum, seed=7)
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
    W0 = [w.float().double() for w in MLP(sizes, net_type, batch=B, momentum=momentum, seed=7).host_weights()]
    for l in range(len(got)):
        dg = got[l] - W0[l]
        dr = W64[l] - W0[l]
        rel = (dg - dr).norm() / (dr.norm() + 1e-30)
        assert rel < 0.05, (l, rel.item())
    lsum, corr = m.read_stats()
    assert lsum == pytest.approx(loss_total * B, rel=0.05)


def test_predict_matches_forward(gpu):
    m = MLP([784, 128, 64, 10], "SNN", batch=128, seed=3)
    X = torch.rand(100, 784, dtype=torch.float64)
    O = m.predict(m.prepare_input(X), n_valid=100).cpu().double()
    R = ref.forward([w.float().bfloat16().double() for w in m.host_weights()], X.float().bfloat16().double(), "SNN")[-1]
    assert (O - R).abs().max().item() < 2e-2
    assert torch.allclose(O.sum(1), torch.ones(100, dtype=torch.float64), atol=1e-4)


@pytest.mark.parametrize("net_type", ["SNN", "ANN", "LNN"])
@pytest.mark.parametrize("B,n_valid", [(1024, 1024), (640, 600)])
def test_fused_matches_layerwise(gpu, net_type, B, n_valid):
    """fused mlp3 path == per-layer path (same math, different summation order)."""
    torch.manual_seed(1)
    sizes = [784, 128, 64, 10]
    mf = MLP(sizes, net_type, batch=B, momentum=True, seed=5, fused=True, mid_grid=3)
    ml = MLP(sizes, net_type, batch=B, momentum=True, seed=5, fused=False)
    assert mf.fused and not ml.fused
    X = torch.rand(mf.Bp, 784)
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
    assert torch.equal(mf.D[0][n_valid:], torch.zeros_like(mf.D[0][n_valid:]))
