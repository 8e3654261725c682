#!/usr/bin/env python3
"""A few launches of the 8-phase NT (forward, bipolar epilogue) and TN GEMMs on
8192x4096x4096, nothing else on the GPU: the program scripts/pmc_8ph.sh profiles."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd import ops  # noqa: E402

B, N, K = 8192, 4096, 4096
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
X = (torch.rand(B, K, device=dev, generator=g) - 0.5).bfloat16()
W = ((torch.rand(N, K, device=dev, generator=g) - 0.5) / 64).bfloat16()
D = ((torch.rand(B, N, device=dev, generator=g) - 0.5) / 8).bfloat16()
out = torch.empty(B, N, dtype=torch.bfloat16, device=dev)
slab = torch.empty(1, N, K, dtype=torch.float32, device=dev)
for _ in range(3):
    ops.gemm_nt(X, W, ops.EPI_ACT, out=out)
    ops.gemm_tn(D, X, splits=1, out=slab)
torch.cuda.synchronize()
print("ok")
