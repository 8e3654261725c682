#!/usr/bin/env python3
"""G0 = delta1^T X weight-gradient GEMM alone (MNIST shape 800x128 over 65536 rows):
median time per launch for several split counts (HPNN_TN_DEEP picks the LDS ring)."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd import ops  # noqa: E402

B = int(os.environ.get("G0_B", "65536"))
X = torch.rand(B, 800, device="cuda").bfloat16()
D = (torch.rand(B, 128, device="cuda") - 0.5).bfloat16()
for S in [int(s) for s in os.environ.get("G0_SPLITS", "32,48,64,96").split(",")]:
    slab = torch.empty(S, 128, 800, device="cuda")
    for _ in range(3):
        ops.gemm_tn(D, X, splits=S, out=slab)
    ts = []
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            ops.gemm_tn(D, X, splits=S, out=slab)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / 20)
    t = statistics.median(ts)
    print(f"deep={os.environ.get('HPNN_TN_DEEP', '-')} splits {S}: {t:.1f} us  X {X.numel() * 2 / t / 1e6:.2f} TB/s")
