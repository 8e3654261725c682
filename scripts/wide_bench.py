#!/usr/bin/env python3
"""Time the wide-input front (ops.wide2_front) alone on the RRUFF shape and, with
HPNN_WIDE_TRACE=1, print the per-phase shader-clock intervals (median / p10 / p90 over
workgroups; s_memtime counts per XCD, so only intervals within a workgroup compare).
usage: [HPNN_WIDE_TRACE=1] python scripts/wide_bench.py [--ksplit 1|2] [--iters N]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd import ops  # noqa: E402
from hpnn_amd._lib import native  # noqa: E402
from hpnn_amd.models import MLP  # noqa: E402

NAMES = ["prologue", "phase A (K slice)", "hand-over", "H0 image + copy-out", "Z = H0 W1^T",
         "output layer", "delta2 copy-out", "delta1", "delta1 copy-out", "stats"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ksplit", type=int, default=0)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=16384)
    a = ap.parse_args()
    B = a.batch
    m = MLP([4096, 230, 230], "SNN", batch=B, momentum=True)
    X = m.prepare_input(torch.rand(B, 4096, device="cuda"))
    lab = torch.randint(0, 230, (B,), device="cuda", dtype=torch.int32)
    ws = ops.Wide2Workspace(B, 4096, "cuda", ksplit=a.ksplit or None)
    outs = [torch.empty(B, 256, dtype=torch.bfloat16, device="cuda") for _ in range(3)]
    run = lambda: ops.wide2_front(X, m.Wb[0], m.Wb[1], m.Wt[1], *outs, ws, 230, ops.TYPE_SNN, labels=lab)  # noqa
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    ws.check()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    flop = 2.0 * B * 256 * 4096
    print(f"wide2_front ksplit={ws.ksplit} batch={B}: {us:.1f} us/launch, layer-0 GEMM {flop / us / 1e6:.0f} TFLOP/s, "
          f"X stream {B * 4096 * 2 / us / 1e6:.2f} TB/s", flush=True)
    if os.environ.get("HPNN_WIDE_TRACE") == "1":
        run()
        torch.cuda.synchronize()
        t = torch.tensor(native().wide2_trace(), dtype=torch.float64).view(512, 12)
        G = min(512, (B // 128) * ws.ksplit)
        t = t[:G]
        for i, name in enumerate(NAMES):
            d = t[:, i + 1] - t[:, i]
            d = d[(t[:, i + 1] > 0) & (t[:, i] > 0)]
            if d.numel() == 0:
                continue
            q = torch.quantile(d, torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64))
            print(f"  {name:24s} n={d.numel():4d} median {q[1]:9.0f}  p10 {q[0]:9.0f}  p90 {q[2]:9.0f} ticks")
        tot = t[:, 10] - t[:, 0]
        fin = tot[t[:, 10] > 0]
        print(f"  whole finisher workgroup median {fin.median():.0f} ticks (shader clock)")


if __name__ == "__main__":
    main()
