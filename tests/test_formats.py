"""File formats (conf / sample / kernel.opt) -- Python side and native C side agree."""
import os

import numpy as np
import pytest

from hpnn_amd.utils import formats


def test_sample_roundtrip(tmp_path):
    x = np.linspace(0, 1, 17)
    t = np.array([1.0, -1.0, -1.0])
    p = tmp_path / "s.txt"
    formats.write_sample(str(p), x, t, comment=0)
    x2, t2 = formats.read_sample(str(p))
    assert np.allclose(x2, x, atol=1e-5) and np.array_equal(t2, t)


def test_kernel_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    ws = [rng.uniform(-1, 1, (8, 4)), rng.uniform(-1, 1, (3, 8))]
    p = tmp_path / "k.opt"
    formats.write_kernel(str(p), ws, name="x", exact=True)
    k = formats.read_kernel(str(p))
    assert k["name"] == "x" and k["sizes"] == [4, 8, 3]
    for a, b in zip(ws, k["weights"]):
        assert np.array_equal(a, b)  # %.17g is exact
    formats.write_kernel(str(p), ws)
    k = formats.read_kernel(str(p))
    for a, b in zip(ws, k["weights"]):
        assert np.abs(a - b).max() < 1e-14  # %17.15f as the reference


def test_conf_roundtrip(tmp_path):
    p = tmp_path / "nn.conf"
    formats.write_conf(str(p), name="t", type="SNN", seed=3, inputs=784, hiddens=[128, 64], outputs=10,
                       train="BPM", batch=256)
    c = formats.read_conf(str(p))
    assert c["type"] == "SNN" and c["hidden"] == [128, 64] and c["input"] == 784 and c["batch"] == 256
    assert c["train"] == "BPM" and c["seed"] == 3
