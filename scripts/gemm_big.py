#!/usr/bin/env python3
"""Large-GEMM throughput of the generic kernels (synthetic 8x4096 ANN shapes) against
torch.matmul (hipBLASLt) on the same shapes: forward NT + bipolar epilogue, backward NT +
f'(h) epilogue, weight-gradient TN.  usage: python scripts/gemm_big.py [--B 8192] [--N 4096]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd import ops  # noqa: E402


def t(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8192)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--K", type=int, default=4096)
    a = ap.parse_args()
    B, N, K = a.B, a.N, a.K
    dev = torch.device("cuda")
    X = (torch.rand(B, K, device=dev) - 0.5).bfloat16()
    W = ((torch.rand(N, K, device=dev) - 0.5) / 64).bfloat16()
    Wt = W.t().contiguous()
    H = (torch.rand(B, N, device=dev) - 0.5).bfloat16()
    D = ((torch.rand(B, N, device=dev) - 0.5) / 8).bfloat16()
    out = torch.empty(B, N, dtype=torch.bfloat16, device=dev)
    dx = torch.empty(B, K, dtype=torch.bfloat16, device=dev)
    fl = 2.0 * B * N * K
    res = {}
    from hpnn_amd._lib import native
    for rnd in range(2):  # interleaved A/B in one process: 1-phase vs 8-phase 256x256 NT kernel
        for mode, tag in ((0, "1ph"), (1, "8ph")):
            native().gemm_nt_set_8ph(1 if mode else 0)
            res[f"nt_fwd_act_{tag}_r{rnd}"] = t(lambda: ops.gemm_nt(X, W, ops.EPI_ACT, out=out))
            res[f"nt_bwd_dact_{tag}_r{rnd}"] = t(lambda: ops.gemm_nt(D, Wt, ops.EPI_DACT, aux=X, out=dx))
    native().gemm_nt_set_8ph(1)
    S = 1
    slab = torch.empty(S, N, K, dtype=torch.float32, device=dev)
    for rnd in range(2):
        for mode, tag in ((0, "4st"), (1, "8ph")):
            native().gemm_tn_set_8ph(mode)
            res[f"tn_grad_{tag}_r{rnd}"] = t(lambda: ops.gemm_tn(D, X, splits=S, out=slab))
    native().gemm_tn_set_8ph(1)
    res["torch_mm_nt"] = t(lambda: torch.matmul(X, W.t()))
    res["torch_mm_tn"] = t(lambda: torch.matmul(D.t(), X))
    for k, v in res.items():
        print(f"{k:22s} {v:9.1f} us  {fl / v / 1e6:8.1f} TFLOP/s")


if __name__ == "__main__":
    main()
