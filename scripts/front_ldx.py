#!/usr/bin/env python3
"""mlp3 front kernel time vs the row pitch of X (800 columns used; pitch 800 = 1600-B rows,
half of them not 128-B aligned; pitch 832 / 864 / 896 = aligned or differently aligned)."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd import ops  # noqa: E402
from hpnn_amd.models import MLP  # noqa: E402

m = MLP([784, 128, 64, 10], "SNN", batch=65536, momentum=True, fused="x")
lab = torch.randint(0, 10, (m.Bp,), device="cuda", dtype=torch.int32)
for pitch in (800, 832, 864, 896, 800):
    Xf = torch.rand(m.Bp, pitch, device="cuda").bfloat16()
    X = Xf[:, :800]
    for _ in range(3):
        m._fused_front(X, lab, None, m.Bp)
    ts = []
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            m._fused_front(X, lab, None, m.Bp)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / 20)
    print(f"pitch {pitch}: front {statistics.median(ts):.1f} us (mode {os.environ.get('HPNN_FZ_MODE', '0')})")
