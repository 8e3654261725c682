#!/usr/bin/env python3
"""Phase timeline of the tile front kernel (HPNN_TILE_TRACE=1 build): median / p10 / p90
over workgroups of the shader-clock intervals between the kernel's phase marks.
usage: HPNN_TILE_TRACE=1 python scripts/tile_trace.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd._lib import native  # noqa: E402
from hpnn_amd.models import MLP  # noqa: E402

NAMES = ["W1 load", "prologue (X(0), W0 ring)", "phase A (25 k-steps)", "H1 epilogue + barrier",
         "chain P1-P4", "phase C (G1, G2)", "slab + stats"]


def main():
    assert os.environ.get("HPNN_TILE_TRACE") == "1"
    dev = torch.device("cuda")
    m = MLP([784, 128, 64, 10], "SNN", batch=65536, momentum=True, fused="t")
    Xs = [m.prepare_input(torch.randint(0, 256, (m.Bp, 784), dtype=torch.uint8, device=dev)) for _ in range(4)]
    lab = torch.randint(0, 10, (m.Bp,), device=dev, dtype=torch.int32)
    for i in range(12):
        m.train_step(Xs[i % 4], labels=lab)
    torch.cuda.synchronize()
    m._fused_front(Xs[1], labels=lab, T=None, n_valid=m.Bp)
    torch.cuda.synchronize()
    G = m.midslab.shape[0]
    t = torch.tensor(native().mlp3_tile_trace(), dtype=torch.float64).view(1024, 8)[:G]
    start = t[:, 0].min()
    print(f"workgroups {G}; kernel span {float(t[:, 7].max() - start):.0f} ticks; "
          f"start skew {float(t[:, 0].max() - start):.0f}")
    for i, n in enumerate(NAMES):
        d = t[:, i + 1] - t[:, i]
        q = torch.quantile(d, torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64))
        print(f"{n:28s} p10 {q[0]:8.0f}  median {q[1]:8.0f}  p90 {q[2]:8.0f} ticks")
    fin = t[:, 7] - start
    print(f"end times: min {float(fin.min()):.0f} median {float(fin.median()):.0f} max {float(fin.max()):.0f}")


if __name__ == "__main__":
    main()
