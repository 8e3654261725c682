#!/bin/bash
# Split-K factor of the G0 GEMM (HPNN_TN_SPLITS), MNIST bench on one GPU, alternating order.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in ${SPLITS:-48 32 40 24 64 48 32 40}; do
  log=gpurun_out/splits_$s.log
  HPNN_TN_SPLITS=$s timeout -k 10 120 python bench.py --steps 400 --warmup 20 > $log 2>&1 || exit 1
  echo "splits=$s $(grep -o '"ms_per_step": [0-9.]*' $log)"
done
