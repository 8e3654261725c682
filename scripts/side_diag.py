#!/usr/bin/env python3
"""RRUFF layer-1 side job vs the separate launches: per-layer max |diff| and differing counts,
plus side-vs-side repeatability (diagnostic).  usage: python scripts/side_diag.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd.models import MLP  # noqa: E402


def run(side, steps=3, B=16384):
    sizes = [4096, 230, 230]
    torch.manual_seed(5)
    m = MLP(sizes, "SNN", batch=B, momentum=True, seed=9)
    m.plan.tn8_side = side
    X = m.prepare_input(torch.rand(B, sizes[0]).cuda())
    for _ in range(steps):
        lab = torch.randint(0, sizes[-1], (B,), dtype=torch.int32, device="cuda")
        m.train_step(X, labels=lab, lr=0.01, alpha=0.2)
    torch.cuda.synchronize()
    return m


def main():
    for steps in (1, 3):
        a, a2, b = run(True, steps), run(True, steps), run(False, steps)
        print(f"steps {steps}: side launches {a.plan.side_launches}/{a2.plan.side_launches}/{b.plan.side_launches}")
        for l in range(2):
            d = (a.W32[l] - b.W32[l]).abs()
            d2 = (a.W32[l] - a2.W32[l]).abs()
            print(f"  layer {l}: side vs sep max {d.max().item():.3e} n {(d > 0).sum().item()}; "
                  f"side vs side max {d2.max().item():.3e} n {(d2 > 0).sum().item()}", flush=True)
            if (d > 0).any():
                idx = (d > 0).nonzero()[:5].tolist()
                print("   first diffs at", idx)


if __name__ == "__main__":
    main()
