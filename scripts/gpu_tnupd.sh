#!/bin/bash
# fused TN + optimizer step: numerics, then the synthetic 8x4096 ANN step with / without it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -x -q -k "tn_update or gemm_tn or train_step" --timeout 120 --timeout-method thread > gpurun_out/tnupd_tests.log 2>&1 || { tail -30 gpurun_out/tnupd_tests.log; exit 1; }
tail -2 gpurun_out/tnupd_tests.log
for rep in 1 2; do
  for u in 1 0; do
    out=$(HPNN_TN_UPD=$u timeout -k 10 300 python scripts/bench_configs.py --only synth_ann --steps 40 2>&1 | grep '{') || exit 1
    echo "tn_upd=$u $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms", round(d["samples_per_s"]), "samples/s", round(d["tflops"]), "TFLOP/s")')" | tee -a gpurun_out/synth_tnupd.txt
  done
done
