#!/usr/bin/env python3
"""Per-kernel timing of the MNIST SNN training step (one process, interleaved reps).

usage: python scripts/kbench.py [--batch 65536] [--reps 50] [--mid-grid 128,256]
Prints one line per phase: median microseconds over reps (HIP events)."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd import ops  # noqa: E402
from hpnn_amd.models import MLP  # noqa: E402


def timeit(fn, reps, inner=20):
    """per-launch time of `inner` back-to-back launches between two events (removes
    the ~8 us event/launch overhead a single-launch measurement carries)."""
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(inner):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / inner)
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--mid-grid", default="512")
    ap.add_argument("--modes", default="x,mid")
    args = ap.parse_args()
    dev = torch.device("cuda")
    for mode in args.modes.split(","):
        m = MLP([784, 128, 64, 10], "SNN", batch=args.batch, momentum=True, fused=mode,
                mid_grid=int(args.mid_grid.split(",")[0]))
        X = m.prepare_input(torch.rand(m.Bp, 784, device=dev))
        lab = torch.randint(0, 10, (m.Bp,), device=dev, dtype=torch.int32)
        bytes_x = X.numel() * 2
        kw = dict(labels=lab, T=None, n_valid=m.Bp)
        phases = {"fused front (" + mode + ")": lambda: m.front(X, **kw)}
        if mode == "mid":
            phases["  fwd_l0 (gemm_nt X.W0^T)"] = lambda: ops.gemm_nt(X, m.Wb[0], ops.EPI_ACT, out=m.H[0])
        phases["grad_l0 (gemm_tn D1^T.X)"] = lambda: ops.gemm_tn(m.D[0], X, splits=m.S[0], out=m.slab[0])
        if mode == "x":
            phases["front + G0 (grads_slabs)"] = lambda: m.grads_slabs(X, **kw)
        phases["full train_step"] = lambda: m.train_step(X, labels=lab)
        for f in phases.values():
            f()
        torch.cuda.synchronize()
        print(f"--- batch {m.Bp} mode {mode} mid slabs {m.midslab.shape[0]} splits {m.S}")
        for name, f in phases.items():
            med, mn = timeit(f, args.reps)
            extra = ""
            if "X" in name:
                extra = f"  X stream {bytes_x / med / 1e6:.2f} TB/s"
            print(f"{name:32s} median {med:8.1f} us  min {mn:8.1f} us{extra}")


if __name__ == "__main__":
    main()
