"""Learnability: the batched BF16 GPU engine (train_nn -m batched, the fused MNIST plan) and
the FP64 CPU batched engine learn the same synthetic task (scripts/learnability.py: noisy
random class prototypes) to the same held-out accuracy.  The full-size record (60000
samples, 8 epochs) is profiles/r4/learnability.jsonl."""
import os
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


@pytest.mark.gpu
def test_bf16_gpu_learns_like_fp64_cpu():
    import learnability as L
    from hpnn_amd import capi
    with tempfile.TemporaryDirectory() as d:
        X, T, _ = L.prototype_data(12800, 1, noise=1.0)
        capi.pack_arrays(os.path.join(d, "train.hpnb"), X, T)
        Xt, Tt, _ = L.prototype_data(2000, 2, noise=1.0)
        capi.pack_arrays(os.path.join(d, "test.hpnb"), Xt, Tt)
        res = {e: L.run(e, d, 3, 0.2, 256, 600) for e in ("gpu", "cpu")}
    g, c = res["gpu"]["test_accuracy"], res["cpu"]["test_accuracy"]
    assert c > 0.9, res["cpu"]
    assert g > 0.9, res["gpu"]
    assert abs(g - c) < 0.03, (g, c)
    # the training loss falls on both
    for r in res.values():
        assert r["epochs"][-1]["loss"] < r["epochs"][0]["loss"]
    assert np.isfinite(res["gpu"]["epochs"][-1]["loss"])
