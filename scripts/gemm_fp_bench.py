"""FP64 / FP32 MFMA GEMM throughput of the reference-precision batched engine
(csrc/gpu/kernels_fp.hip gemm_fp) against the matrix-core peaks (MI355X: FP64 78.6 TF,
FP32 157.3 TF, dense) and torch.matmul (hipBLASLt / rocBLAS) on the same shapes.

    python scripts/gemm_fp_bench.py [--out file.jsonl]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd._lib import native  # noqa: E402

PEAK = {"f64": 78.6e12, "f32": 157.3e12}


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    n = native()
    s = torch.cuda.current_stream().cuda_stream
    # (M, N, K, ta, tb): forward X W^T (NT), delta GEMM D W (NN on W), weight gradient D^T H (TT)
    shapes = [(8192, 4096, 4096, 0, 0), (8192, 4096, 4096, 0, 1), (4096, 4096, 8192, 1, 1),
              (16384, 256, 4096, 0, 0), (65536, 128, 784, 0, 0)]
    for dt, tdt in (("f64", torch.float64), ("f32", torch.float32)):
        for M, N, K, ta, tb in shapes:
            A = torch.randn(K, M, dtype=tdt, device="cuda") if ta else torch.randn(M, K, dtype=tdt, device="cuda")
            B = torch.randn(K, N, dtype=tdt, device="cuda") if tb else torch.randn(N, K, dtype=tdt, device="cuda")
            C = torch.empty(M, N, dtype=tdt, device="cuda")

            def ours():
                n.gemm_fp(int(dt == "f64"), A.data_ptr(), A.stride(0), ta, B.data_ptr(), B.stride(0), tb,
                          C.data_ptr(), C.stride(0), 0, 0, M, N, K, 0, 1, 0, s)
            t = timed(ours, a.reps)
            Am = A.t() if ta else A
            Bm = B if tb else B.t()
            ref = Am @ Bm
            err = ((C - ref).abs().max() / ref.abs().max()).item()
            tt = timed(lambda: torch.matmul(Am, Bm), a.reps)
            fl = 2.0 * M * N * K
            rec = {"dtype": dt, "M": M, "N": N, "K": K, "ta": ta, "tb": tb, "us": round(t * 1e6, 1),
                   "tflops": round(fl / t / 1e12, 2), "pct_peak": round(100 * fl / t / PEAK[dt], 1),
                   "torch_us": round(tt * 1e6, 1), "torch_tflops": round(fl / tt / 1e12, 2), "max_rel_err": err}
            print(json.dumps(rec), flush=True)
            if a.out:
                with open(a.out, "a") as f:
                    f.write(json.dumps(rec) + "\n")
            del A, B, C, ref


if __name__ == "__main__":
    main()
