"""The plan's choice of step structure (csrc/gpu/bplan.cpp BPlan::configure, the one the
C engine and hpnn_amd.models.MLP share), checked without a GPU."""
import pytest
import torch

from hpnn_amd.models import MLP


def test_wide_mode_selected_for_the_rruff_shape():
    m = MLP([4096, 230, 230], "SNN", batch=256, device="cpu")
    assert m.fused_mode == "w" and m.cfg["input_layout"] == 0
    assert MLP([4000, 230, 230], "SNN", batch=256, device="cpu").fused_mode is None
    with pytest.raises(ValueError):
        MLP([4000, 230, 230], "SNN", batch=256, device="cpu", fused="w")


@pytest.mark.parametrize("batch,mode,Bp", [(65536, "t", 65536), (256, "t", 256), (384, "x", 384), (100, "x", 128)])
def test_mnist_shape_modes(batch, mode, Bp):
    """the 256-sample tile front when the padded batch is whole tiles, else the 32-sample
    pipelined front; an explicit tile request pads the batch to whole tiles"""
    m = MLP([784, 128, 64, 10], "SNN", batch=batch, device="cpu")
    assert (m.fused_mode, m.Bp) == (mode, Bp)
    assert m.cfg["buckets"] == [(1, 2), (0, 0)]
    t = MLP([784, 128, 64, 10], "SNN", batch=100, device="cpu", fused="t")
    assert t.fused_mode == "t" and t.Bp == 256
    assert MLP([784, 128, 64, 10], "SNN", batch=256, device="cpu", fused=False).fused_mode is None
    assert MLP([32, 128, 64, 10], "SNN", batch=256, device="cpu").fused_mode == "mid"


def test_cpu_emulation_trains_in_any_mode():
    """on CPU tensors every mode runs the per-layer emulation: same result"""
    torch.manual_seed(0)
    X = torch.rand(256, 784)
    lab = torch.randint(0, 10, (256,), dtype=torch.int32)
    ms = [MLP([784, 128, 64, 10], "SNN", batch=256, device="cpu", momentum=True, seed=7, fused=f) for f in (None, False)]
    for m in ms:
        m.train_step(m.prepare_input(X), labels=lab, lr=0.05, alpha=0.2)
    for a, b in zip(ms[0].host_weights(), ms[1].host_weights()):
        assert torch.equal(a, b)
