#!/usr/bin/env python3
"""Per-interval timeline of mlp3_fused (HPNN_FZ_MODE=9 build-in instrumentation)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd._lib import native  # noqa: E402
from hpnn_amd.models import MLP  # noqa: E402

assert os.environ.get("HPNN_FZ_MODE") in ("9", "10", "11")
m = MLP([784, 128, 64, 10], "SNN", batch=65536, momentum=True, fused="x")
X = m.prepare_input(torch.rand(m.Bp, 784, device="cuda"))
lab = torch.randint(0, 10, (m.Bp,), device="cuda", dtype=torch.int32)
for _ in range(5):
    m._fused_front(X, lab, None, m.Bp)
torch.cuda.synchronize()
NW = 8  # both kernels: 8 waves (mlp3_front: 0-3 front, 4-7 back)
tr = torch.tensor(native().mlp3_fused_trace(), dtype=torch.float64).view(8, 8, 8)
t0 = tr[:NW, 0, 0].min()
tr = tr - t0
print("ticks relative to wave min at stage 0 mark 0; marks: [end I3 prev | after B0 | end I0 | after B1 | end I1 | after B2 | end I2 | after B3]")
for w in (0, 4, 5):
    for t in range(7):
        print(f"w{w} s{t}: " + " ".join(f"{int(v):7d}" for v in tr[w, t]))
# per-interval durations averaged over stages 2..6, per wave
print("interval work (end - after barrier) and wait (after next barrier - end), stages 2-5 mean:")
for w in range(NW):
    works, waits = [], []
    for j in range(4):
        wk = (tr[w, 2:6, 2 * j + 2] if j < 3 else tr[w, 3:7, 0]) - tr[w, 2:6, 2 * j + 1]
        works.append(wk.mean().item())
    st = (tr[w, 3:7, 1] - tr[w, 2:6, 1]).mean().item()
    print(f"w{w}: work I0..I3 = " + " ".join(f"{x:6.0f}" for x in works) + f"   stage = {st:6.0f}")
if os.environ.get("HPNN_FRONT", "") == "f":  # mlp3_front: 2 intervals per stage, kernel marks
    raw = torch.tensor(native().mlp3_fused_trace(), dtype=torch.float64).view(8, 8, 8)
    print("mlp3_front: per-wave work of interval 0 / 1 and stage length (stages 2-5 mean)")
    for w in range(8):
        i0 = (raw[w, 2:6, 2] - raw[w, 2:6, 1]).mean().item()
        i1 = (raw[w, 3:7, 0] - raw[w, 2:6, 3]).mean().item()
        st = (raw[w, 3:7, 1] - raw[w, 2:6, 1]).mean().item()
        print(f"w{w}: I0 {i0:6.0f}  I1 {i1:6.0f}  stage {st:6.0f}")
    t0 = raw[:, 7, 0].min()
    for w in range(8):
        e = raw[w, 7, :3] - t0
        print(f"w{w}: prologue done {int(e[1])}  first barrier passed {int(raw[w, 0, 1] - t0)}  "
              f"loop end {int(e[2])} (ticks from the first entry)")
