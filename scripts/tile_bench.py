#!/usr/bin/env python3
"""Per-kernel times of the MNIST SNN step (batch 65536, 8-bit pixels) on the fused front
paths: "x" (mlp3_fused, 32-sample pipelined tiles) and "t" (mlp3_tile, 256-sample tiles).
usage: python scripts/tile_bench.py [--modes t,x] [--reps 10]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd.models import MLP  # noqa: E402
from scripts.kbench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--modes", default="t,x")
    ap.add_argument("--sets", type=int, default=4, help="distinct batches cycled (cold HBM reads)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    for mode in args.modes.split(","):
        m = MLP([784, 128, 64, 10], "SNN", batch=args.batch, momentum=True, fused=mode)
        Xs = [m.prepare_input(torch.randint(0, 256, (m.Bp, 784), dtype=torch.uint8, device=dev))
              for _ in range(args.sets)]
        lab = torch.randint(0, 10, (m.Bp,), device=dev, dtype=torch.int32)
        kw = dict(labels=lab, T=None, n_valid=m.Bp)
        it = [0]

        def nxt():
            it[0] += 1
            return Xs[it[0] % len(Xs)]
        phases = {
            f"front ({mode})": lambda: m.front(nxt(), **kw),
            "front + G0 (grads_slabs)": lambda: m.grads_slabs(nxt(), **kw),
            "full train_step": lambda: m.train_step(nxt(), labels=lab),
        }
        for f in phases.values():
            f()
        torch.cuda.synchronize()
        print(f"--- batch {m.Bp} mode {mode} grid {m.midslab.shape[0]} splits {m.S}")
        for name, f in phases.items():
            med, mn = timeit(f, args.reps)
            print(f"{name:30s} median {med:8.1f} us  min {mn:8.1f} us")


if __name__ == "__main__":
    main()
