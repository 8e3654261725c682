#!/bin/bash
# split-K 8-phase NT: numerics, then the RRUFF-shaped step with / without it (alternating).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "nt8 or big_tile or gemm_nt or gemm_tn" --timeout 120 --timeout-method thread > gpurun_out/splitk_tests.log 2>&1 || { tail -30 gpurun_out/splitk_tests.log; exit 1; }
tail -2 gpurun_out/splitk_tests.log
for rep in 1 2; do
  for m in 1 0; do
    out=$(HPNN_NT_8PH=$m timeout -k 10 200 python scripts/bench_configs.py --only rruff_snn --steps 200 2>&1 | grep '{') || exit 1
    echo "nt8=$m $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,1), "us", round(d["tflops"]), "TFLOP/s")')" | tee -a gpurun_out/rruff_splitk.txt
  done
done
