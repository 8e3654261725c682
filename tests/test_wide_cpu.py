"""The wide-input front (mode "w", csrc/gpu/kernels_wide.hip) on CPU tensors: its PyTorch
emulation drives the same training step as the per-layer path (the GPU kernel is checked
against this emulation in tests/test_wide_gpu.py)."""
import pytest
import torch

from hpnn_amd import ops
from hpnn_amd.models import MLP


@pytest.mark.parametrize("net,labels", [("SNN", True), ("ANN", False)])
def test_wide_mode_step_equals_layerwise_on_cpu(net, labels):
    torch.manual_seed(0)
    B, sizes = 200, [4096, 230, 230]
    mw = MLP(sizes, net, batch=B, device="cpu", momentum=True, seed=7, fused="w")
    ml = MLP(sizes, net, batch=B, device="cpu", momentum=True, seed=7, fused=False)
    assert mw.fused_mode == "w" and ml.fused_mode is None
    X = torch.rand(B, sizes[0])
    lab = torch.randint(0, sizes[-1], (B,), dtype=torch.int32)
    kw = {}
    if labels:
        kw["labels"] = torch.cat([lab, torch.zeros(mw.Bp - B, dtype=torch.int32)])
    else:
        T = torch.full((mw.Bp, sizes[-1]), -1.0)
        T[torch.arange(B), lab.long()] = 1.0
        kw["T"] = T
    for _ in range(2):
        mw.train_step(mw.prepare_input(X), n_valid=B, lr=0.05, alpha=0.2, **kw)
        ml.train_step(ml.prepare_input(X), n_valid=B, lr=0.05, alpha=0.2, **kw)
    for a, b in zip(mw.host_weights(), ml.host_weights()):
        assert torch.equal(a, b)
    assert mw.read_stats() == ml.read_stats()


def test_wide_mode_selected_for_the_rruff_shape():
    m = MLP([4096, 230, 230], "SNN", batch=256, device="cpu")
    assert m.fused_mode == "w"
    assert MLP([4000, 230, 230], "SNN", batch=256, device="cpu").fused_mode is None
    assert ops.WIDE2_TILE == 128
