#!/bin/bash
# 8-phase NT GEMM: numerics (direct + dispatched big-tile shapes), in-process A/B against
# the 1-phase 256x256 kernel, then the synthetic 8x4096 ANN config with each kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "nt8 or big_tile or gemm_nt or gemm_tn" --timeout 120 --timeout-method thread > gpurun_out/nt8_tests.log 2>&1 || { tail -30 gpurun_out/nt8_tests.log; exit 1; }
tail -2 gpurun_out/nt8_tests.log
timeout -k 10 200 python scripts/gemm_big.py 2>&1 | tee gpurun_out/nt8_gemm_big.txt || exit 1
for mode in 1 0 1 0; do
  HPNN_NT_8PH=$mode HPNN_TN_8PH=$mode timeout -k 10 300 python scripts/bench_configs.py --only synth_ann 2>&1 | grep '{' | sed "s/^/nt8=$mode /" | tee -a gpurun_out/nt8_synth.txt || exit 1
done
