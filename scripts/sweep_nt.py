#!/usr/bin/env python3
"""Time gemm_nt (X[M x K] . W[N x K]^T, bipolar epilogue) over M: separates the fixed
per-launch cost from the streaming rate.  usage: python scripts/sweep_nt.py [K] [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd import ops  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 800
N = int(sys.argv[2]) if len(sys.argv) > 2 else 128
tag = "generic" if os.environ.get("HPNN_NO_WS") == "1" else "ws"
for M in (8192, 16384, 32768, 65536, 131072, 262144):
    nbuf = max(1, (400 << 20) // (M * K * 2))  # rotate buffers so X is not cache-resident
    Xs = [torch.rand(M, K, device="cuda").bfloat16() for _ in range(nbuf)]
    W = torch.rand(N, K, device="cuda").bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    it = [0]

    def f():
        ops.gemm_nt(Xs[it[0] % nbuf], W, ops.EPI_ACT, out=C)
        it[0] += 1
    f()
    med, mn = timeit(f, 10, inner=nbuf * 4)
    print(f"{tag} K={K} N={N} M={M:7d} nbuf={nbuf}: {med:8.1f} us  X {M * K * 2 / med / 1e6:5.2f} TB/s")
    del Xs
