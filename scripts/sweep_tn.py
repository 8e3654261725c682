#!/usr/bin/env python3
"""gemm_tn (G0 = D1^T X, MNIST shape) time vs split count; X rotated over 4 buffers."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd import ops  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

B, N, M = 65536, 128, 800
Xs = [torch.rand(B, M, device="cuda").bfloat16() for _ in range(4)]
D = (torch.rand(B, N, device="cuda") - 0.5).bfloat16()
for S in (16, 32, 64, 128):
    slab = torch.empty(S, N, M, device="cuda")
    it = [0]

    def f():
        ops.gemm_tn(D, Xs[it[0] % 4], splits=S, out=slab)
        it[0] += 1
    f()
    med, mn = timeit(f, 10, inner=8)
    print(f"S={S:4d} grid={5 * S:4d}: {med:7.1f} us (min {mn:7.1f})  slab {S * N * M * 4 / 1e6:6.1f} MB")
