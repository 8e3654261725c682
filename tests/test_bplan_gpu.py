"""One orchestrator: train_nn's batched BF16 engine (gpu_engine.cpp, C) and
hpnn_amd.models.MLP (Python) drive the SAME plan (csrc/gpu/bplan.h) -- same step structure,
split counts and kernels -- so three minibatch steps give the same weights bit for bit.
Reference entry point being replaced: tests/train_nn.c:232 -> nn_train_kernel
(libhpnn.c:1149-1302)."""
import ctypes
import ctypes.util
import os
import subprocess

import numpy as np
import pytest
import torch

from hpnn_amd.models import MLP
from hpnn_amd.utils import formats

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


def _order(n, seed):
    """nn_train_kernel's seeded sample order (api.cpp seeded_order, libhpnn.c:1218-1229)"""
    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    libc.random.restype = ctypes.c_long
    libc.srandom(ctypes.c_uint(seed))
    used, order = set(), []
    while len(order) < n:
        idx = int(float(libc.random()) * n / 2147483647.0)
        if idx >= n or idx in used:
            continue
        used.add(idx)
        order.append(idx)
    return order


@pytest.mark.gpu
@pytest.mark.parametrize("net,train,dims,B,pixels,mode", [
    ("SNN", "BPM", (784, [128, 64], 10), 256, True, "t"),     # tile front, 8-bit input
    ("SNN", "BPM", (784, [128, 64], 10), 384, True, "x"),     # pipelined front + byte copy for G0
    ("SNN", "BPM", (4096, [230], 230), 256, False, "w"),      # wide front
    ("ANN", "BP", (100, [64, 48], 7), 128, False, None),      # per-layer kernels
])
def test_train_nn_batched_equals_python_plan(tmp_path, gpu, net, train, dims, B, pixels, mode):
    n_in, hid, n_out = dims
    n, seed, steps = 3 * B, 11, 3
    rng = np.random.default_rng(5)
    X = rng.integers(0, 256, (n, n_in)).astype(np.float64) if pixels else rng.uniform(-1, 1, (n, n_in))
    lab = rng.integers(0, n_out, n)
    T = np.full((n, n_out), 0.0 if net == "SNN" else -1.0)
    T[np.arange(n), lab] = 1.0
    from hpnn_amd import capi
    d = str(tmp_path)
    capi.pack_arrays(os.path.join(d, "train.hpnb"), X, T)
    formats.write_conf(os.path.join(d, "nn.conf"), name="t", type=net, seed=seed, inputs=n_in, hiddens=hid,
                       outputs=n_out, train=train, sample_dir="./train.hpnb", test_dir="./train.hpnb",
                       mode="batched", batch=B, epochs=1, dtype="bf16", lr=0.01)
    env = dict(os.environ)
    env.pop("HPNN_FORCE_CPU", None)
    r = subprocess.run([os.path.join(BIN, "train_nn"), "-vvv", "nn.conf"], cwd=d, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"batched plan: mode {mode or '-'}" in r.stdout, r.stdout[-3000:]
    got = formats.read_kernel(os.path.join(d, "kernel.opt"))["weights"]

    m = MLP([n_in] + hid + [n_out], net, batch=B, momentum=train == "BPM", seed=seed)
    assert m.fused_mode == {"t": "t", "x": "x", "w": "w", None: None}[mode]
    tmp = formats.read_kernel(os.path.join(d, "kernel.tmp"))["weights"]
    for a, b in zip(tmp, m.host_weights()):
        # same seeded init (ann.c:632-766); the plan keeps FP32 masters
        assert np.abs(a - b.numpy()).max() <= 2.0 ** -24 * np.abs(a).max()
    order = _order(n, seed)
    Xo, To = X[order], T[order]
    for s in range(steps):
        xb = torch.tensor(Xo[s * B:(s + 1) * B])
        xb = xb.to(torch.uint8) if pixels else xb  # the bytes ARE the values (scale 1), as train_nn
        Xp = m.prepare_input(xb, pixel_scale=1.0)
        Tt = torch.tensor(To[s * B:(s + 1) * B], dtype=torch.float32, device="cuda")
        Tt = torch.cat([Tt, torch.zeros(m.Bp - B, n_out, device="cuda")]) if m.Bp > B else Tt
        m.train_step(Xp, T=Tt.contiguous(), n_valid=B, lr=0.01, alpha=0.2 if train == "BPM" else 0.0)
    torch.cuda.synchronize()
    for a, w in zip(got, m.W32):
        ref = w[:a.shape[0], :a.shape[1]].double().cpu().numpy()
        # kernel.opt prints 15 decimals: recovers every FP32 master weight exactly
        assert np.array_equal(a.astype(np.float32).astype(np.float64), ref), np.abs(a - ref).max()
