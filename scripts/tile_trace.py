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

NAMES = ["W1 DMA issue", "prologue (X(0), W0 ring)", "phase A (25 k-steps)", "H1 epilogue + barrier",
         "P1 (H2)", "P2 (output, loss, delta3)", "P3 (delta2)", "P4 (delta1 -> HBM) + barrier",
         "phase C (G1, G2)", "slab + stats"]


def main():
    assert os.environ.get("HPNN_TILE_TRACE") == "1"
    nd = int(sys.argv[1]) if len(sys.argv) > 1 else 4  # distinct batches cycled (1: X stays in the Infinity Cache)
    dev = torch.device("cuda")
    m = MLP([784, 128, 64, 10], "SNN", batch=65536, momentum=True, fused="t")
    Xs = [m.prepare_input(torch.randint(0, 256, (m.Bp, 784), dtype=torch.uint8, device=dev)) for _ in range(nd)]
    lab = torch.randint(0, 10, (m.Bp,), device=dev, dtype=torch.int32)
    for i in range(12):
        m.train_step(Xs[i % nd], labels=lab)
    torch.cuda.synchronize()
    m._fused_front(Xs[1 % nd], labels=lab, T=None, n_valid=m.Bp)
    torch.cuda.synchronize()
    G = m.midslab.shape[0]
    t = torch.tensor(native().mlp3_tile_trace(), dtype=torch.float64).view(1024, 12)[:G]
    tot = t[:, 10] - t[:, 0]
    print(f"workgroups {G}; per-workgroup span median {float(tot.median()):.0f} ticks "
          f"(s_memtime is per XCD: only intervals within a workgroup are compared)")
    for i, n in enumerate(NAMES):
        d = t[:, i + 1] - t[:, i]
        q = torch.quantile(d, torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64))
        print(f"{n:28s} p10 {q[0]:8.0f}  median {q[1]:8.0f}  p90 {q[2]:8.0f} ticks")



if __name__ == "__main__":
    main()
