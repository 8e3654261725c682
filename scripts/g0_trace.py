#!/usr/bin/env python3
"""Phase timeline of the fused first-layer-gradient launch (HPNN_G0_TRACE=1): median / p10 /
p90 over workgroups of the shader-clock intervals between its phase marks, and each phase's
END relative to the earliest workgroup start on the same XCD (s_memtime is per XCD).
usage: HPNN_G0_TRACE=1 python scripts/g0_trace.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd._lib import native  # noqa: E402
from hpnn_amd.models import MLP  # noqa: E402

NAMES = ["GEMM (fm_partial, K split)", "publish partials + ticket", "[G1|G2] share + layer 1/2 steps",
         "wait for the tile's splits", "reduce 1/splits of the tile + layer-0 step"]


def main():
    assert os.environ.get("HPNN_G0_TRACE") == "1"
    dev = torch.device("cuda")
    m = MLP([784, 128, 64, 10], "SNN", batch=65536, momentum=True, fused="t")
    Xs = [m.prepare_input(torch.randint(0, 256, (m.Bp, 784), dtype=torch.uint8, device=dev)) for _ in range(4)]
    lab = torch.randint(0, 10, (m.Bp,), device=dev, dtype=torch.int32)
    for i in range(12):
        m.train_step(Xs[i % 4], labels=lab)
    torch.cuda.synchronize()
    import ctypes
    from hpnn_amd._lib import lib_path
    G = ctypes.CDLL(lib_path()).hpnn_g0_tiles(1, m.Np[0], m.Kp[0]) * m.S[0]
    ta = torch.tensor(native().g0_trace(), dtype=torch.float64).view(512, 8)
    t = ta[:G]
    print(f"workgroups {G}; span median {float((t[:, 5] - t[:, 0]).median()):.0f} ticks")
    # tail workgroups (blocks G..: the [G1 | G2] share beside the GEMM): start -> done
    tail = ta[G:256]
    tail = tail[tail[:, 6] > tail[:, 0]]
    if len(tail):
        d = tail[:, 6] - tail[:, 0]
        print(f"tail workgroups {len(tail)}: [G1|G2] share (+ exchange) median {float(d.median()):.0f}  "
              f"max {float(d.max()):.0f} ticks (GEMM workgroups' span median "
              f"{float((t[:, 5] - t[:, 0]).median()):.0f})")
    for i, n in enumerate(NAMES):
        d = t[:, i + 1] - t[:, i]
        q = torch.quantile(d, torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64))
        print(f"{n:44s} p10 {q[0]:8.0f}  median {q[1]:8.0f}  p90 {q[2]:8.0f} ticks")
    # per XCD (blocks b, b + 8, ... share one under round-robin placement): phase ends after
    # the XCD's first workgroup start
    ends = []
    for x in range(8):
        tx = t[x::8]
        ends.append(tx[:, 1:6] - tx[:, 0].min())
    e = torch.cat(ends)
    med = e.median(dim=0).values
    mx = e.max(dim=0).values
    print("phase end after the XCD's first start (median / max): " +
          ", ".join(f"{a:.0f}/{b:.0f}" for a, b in zip(med.tolist(), mx.tolist())))


if __name__ == "__main__":
    main()
