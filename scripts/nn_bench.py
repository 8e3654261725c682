#!/usr/bin/env python3
"""The sharded step's delta GEMM alone at the 8-GPU shard shape (1024 x 4096 x 4096): NN form
(W read directly, hpnn_gemm_nn_bf16) vs the NT form on W^T, each epilogue; plus the transpose
the NN form saves.  usage: python scripts/nn_bench.py [--M 1024]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd import ops  # noqa: E402
from hpnn_amd._lib import native  # noqa: E402


def timeit(fn, reps=10, inner=20):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(inner):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / inner)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=1024)
    a = ap.parse_args()
    M, N, K = a.M, 4096, 4096
    A = (torch.rand(M, K, device="cuda") - 0.5).bfloat16()
    W = (torch.rand(K, N, device="cuda") - 0.5).bfloat16()
    Wt = W.t().contiguous()
    aux = (torch.rand(M, N, device="cuda") - 0.5).bfloat16()
    C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    flop = 2.0 * M * N * K
    for epi, name in ((ops.EPI_ACT, "act"), (ops.EPI_DACT, "dact")):
        x = aux if epi == ops.EPI_DACT else None
        nt = timeit(lambda: ops.gemm_nt(A, Wt, epi, aux=x, out=C))
        nn = timeit(lambda: native().gemm_nn_bf16(A.data_ptr(), K, W.data_ptr(), N, C.data_ptr(), N,
                                                  aux.data_ptr(), N, M, N, K, epi, 0, s))
        print(f"{name}: NT on W^T {nt:6.1f} us ({flop / nt / 1e6:5.0f} TFLOP/s), NN on W {nn:6.1f} us "
              f"({flop / nn / 1e6:5.0f} TFLOP/s)", flush=True)
    T = torch.empty_like(W)
    tr = timeit(lambda: native().transpose_bf16(W.data_ptr(), T.data_ptr(), K, N, s))
    print(f"transpose_bf16 4096 x 4096: {tr:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
