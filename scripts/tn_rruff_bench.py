#!/usr/bin/env python3
"""RRUFF first-layer weight gradient G0 = D1^T X (256 x 4096 over 16384 rows) alone:
the 8-phase TN kernel at several split-K factors (FP32 slabs), the slab sum, and the
library GEMM (torch.matmul -> hipBLASLt, BF16 out) on the same operands as a yardstick.
usage: python scripts/tn_rruff_bench.py [--rows 16384] [--splits 8,16,32]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd import ops  # noqa: E402


def timeit(fn, reps=10, inner=20):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(inner):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / inner)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16384)
    ap.add_argument("--splits", default="8,16,32")
    a = ap.parse_args()
    B, N, M = a.rows, 256, 4096
    g = torch.Generator(device="cuda").manual_seed(0)
    D = (torch.rand(B, N, device="cuda", generator=g) - 0.5).bfloat16()
    H = torch.rand(B, M, device="cuda", generator=g).bfloat16()
    flop = 2.0 * B * N * M
    ref = D.float().t() @ H.float()
    for s in [int(v) for v in a.splits.split(",")]:
        out = torch.empty(s, N, M, device="cuda")
        us = timeit(lambda: ops.gemm_tn(D, H, splits=s, out=out))
        err = ((out.sum(0) - ref).abs().max() / ref.abs().max()).item()
        red = torch.empty(N, M, device="cuda")
        us_r = timeit(lambda: torch.sum(out, 0, out=red))
        print(f"gemm_tn splits={s:3d}: {us:7.1f} us ({flop / us / 1e6:6.0f} TFLOP/s), slabs {s * N * M * 4 / 1e6:.0f} MB, "
              f"torch.sum of slabs {us_r:6.1f} us, rel err {err:.1e}", flush=True)
    Dt = D.t()
    us = timeit(lambda: torch.matmul(Dt, H))
    print(f"torch.matmul D^T H (hipBLASLt, bf16 out): {us:7.1f} us ({flop / us / 1e6:6.0f} TFLOP/s)", flush=True)
    Xs = torch.empty(B, M, dtype=torch.bfloat16, device="cuda")
    us = timeit(lambda: Xs.copy_(H))
    print(f"copy of X ({B * M * 2 / 1e6:.0f} MB read + write): {us:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
