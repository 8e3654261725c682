#!/usr/bin/env python3
"""Loss trajectories of the three batched-training paths on the same synthetic data
(consistency check of the fused kernels over many steps)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd.models import MLP  # noqa: E402

B, steps = int(os.environ.get("B", 65536)), int(os.environ.get("STEPS", 240))
g = torch.Generator(device="cuda").manual_seed(1234)
data = None
for mode in ("x", "mid", False):
    m = MLP([784, 128, 64, 10], "SNN", batch=B, momentum=True, seed=10958, fused=mode)
    if data is None:
        data = [(m.prepare_input(torch.rand(m.Bp, 784, device="cuda", generator=g)),
                 torch.randint(0, 10, (m.Bp,), device="cuda", generator=g, dtype=torch.int32)) for _ in range(4)]
    line = []
    for i in range(steps):
        if i % 40 == 0:
            m.reset_stats()
        X, L = data[i % 4]
        m.train_step(X, labels=L, lr=0.01, alpha=0.2)
        if i % 40 == 39:
            ls, c = m.read_stats()
            line.append(f"{ls / (40 * m.Bp):.5f}/{c / (40 * m.Bp):.4f}")
    print(f"mode={mode!s:5s} loss/acc per 40 steps:", " ".join(line), flush=True)
