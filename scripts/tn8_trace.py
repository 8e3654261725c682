#!/usr/bin/env python3
"""RRUFF step with HPNN_TN8_TRACE=1: per-phase shader-clock intervals of the layer-0 fused TN
launch (kernels_8ph.hip MODE 2, with layer 1's side job): median / p10 / p90 over workgroups.
usage: HPNN_TN8_TRACE=1 python scripts/tn8_trace.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd._lib import native  # noqa: E402
from hpnn_amd.models import MLP  # noqa: E402

NAMES = ["side pieces + arrive", "layer-0 GEMM", "publish + arrive", "side wait", "side reduce + step",
         "tile wait", "layer-0 reduce + step"]


def main():
    B = 16384
    m = MLP([4096, 230, 230], "SNN", batch=B, momentum=True)
    X = m.prepare_input(torch.rand(B, 4096, device="cuda"))
    for _ in range(20):
        lab = torch.randint(0, 230, (B,), dtype=torch.int32, device="cuda")
        m.train_step(X, labels=lab, lr=0.01, alpha=0.2)
    torch.cuda.synchronize()
    print(f"side launches {m.plan.side_launches}, splits {list(m.S)}", flush=True)
    t = torch.tensor(native().tn8_trace(), dtype=torch.float64).view(512, 8)
    t = t[(t[:, 0] > 0)]
    for i, name in enumerate(NAMES):
        d = t[:, i + 1] - t[:, i]
        d = d[(t[:, i + 1] > 0) & (t[:, i] > 0)]
        if d.numel() == 0:
            continue
        q = torch.quantile(d, torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64))
        print(f"  {name:24s} n={d.numel():4d} median {q[1]:9.0f}  p10 {q[0]:9.0f}  p90 {q[2]:9.0f} ticks")
    tot = (t[:, 7] - t[:, 0])[t[:, 7] > 0]
    print(f"  whole workgroup median {tot.median():.0f} ticks (shader clock)")


if __name__ == "__main__":
    main()
