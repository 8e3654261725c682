#!/bin/bash
# 8-phase NT on 32x32x16 vs 16x16x32 MFMAs: numerics, in-process GEMM A/B, synthetic step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "nt8" --timeout 120 --timeout-method thread > gpurun_out/m32_tests.log 2>&1 || { tail -30 gpurun_out/m32_tests.log; exit 1; }
tail -2 gpurun_out/m32_tests.log
timeout -k 10 200 python scripts/gemm_big.py 2>&1 | grep -v amdgpu | tee gpurun_out/m32_gemm_big.txt || exit 1
for rep in 1 2; do
  for m in 1 0; do
    out=$(HPNN_NT8_M32=$m timeout -k 10 300 python scripts/bench_configs.py --only synth_ann --steps 40 2>&1 | grep '{') || exit 1
    echo "m32=$m $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms", round(d["tflops"]), "TFLOP/s")')" | tee -a gpurun_out/m32_synth.txt
  done
done
