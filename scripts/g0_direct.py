#!/usr/bin/env python3
"""MNIST first-layer weight gradient (800 x 128 over 65536 rows) with the TN kernels:
LDS-DMA pipe (ops.gemm_tn), register-staged (ops.gemm_tn_rs; rs-u8: the input as 8-bit
pixels, converted while staging), fragment-major direct loads (ops.gemm_fm_direct).  "hot": the same operands every call (they stay in the 256 MB MALL);
"cold": cycling over 4 operand sets (420 MB, from HBM).  usage: g0_direct.py [splits]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd import ops  # noqa: E402


def t(fn, n, reps=48):
    for i in range(4):
        fn(i % n)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(reps):
        fn(i % n)
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


B, M, N = 65536, 800, 128
S = int(sys.argv[1]) if len(sys.argv) > 1 else 48
dev = torch.device("cuda")
Xu = [torch.randint(0, 256, (B, M), device=dev, dtype=torch.uint8) for _ in range(4)]  # pixel values
Xs = [x.bfloat16() for x in Xu]  # exact
Ds = [((torch.rand(B, N, device=dev) - 0.5) / 8).bfloat16() for _ in range(4)]
Xg = [ops.to_fragment_major(x) for x in Xs]
Dg = [ops.to_fragment_major(d) for d in Ds]
Xgu = [ops.to_fragment_major(x) for x in Xu]
out = torch.empty(S, N, M, device=dev)
ref = Ds[0].float().t() @ Xs[0].float()
for name, fn in [("tn", lambda i: ops.gemm_tn(Ds[i], Xs[i], splits=S, out=out)),
                 ("rs", lambda i: ops.gemm_tn_rs(Ds[i], Xs[i], splits=S, out=out)),
                 ("fm", lambda i: ops.gemm_fm_direct(Dg[i], Xg[i], N, M, splits=S, out=out)),
                 ("rs-u8", lambda i: ops.gemm_tn_rs(Ds[i], Xu[i], splits=S, out=out)),
                 ("fm-u8", lambda i: ops.gemm_fm_direct(Dg[i], Xgu[i], N, M, splits=S, out=out))]:
    hot, cold = t(fn, 1), t(fn, 4)
    fn(0)
    err = (out.sum(0) - ref).abs().max().item()
    print(f"splits {S} {name}: hot {hot:6.1f} us  cold {cold:6.1f} us  err {err:.2e} (|ref| max {ref.abs().max().item():.1f})")
