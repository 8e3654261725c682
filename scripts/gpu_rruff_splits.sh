#!/bin/bash
# RRUFF-shaped SNN step vs the weight-gradient split count (16 routes G0 to the 8-phase TN kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for rep in 1 2; do
  for s in 0 8 16 32; do
    out=$(HPNN_TN_SPLITS=$s timeout -k 10 200 python scripts/bench_configs.py --only rruff_snn --steps 200 2>&1 | grep '{') || exit 1
    echo "splits=$s $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,1), "us")')" | tee -a gpurun_out/rruff_splits.txt
  done
done
