#!/bin/bash
# bench A/B: W0 prologue overlapped with stage 0 (default) vs full wait (HPNN_FZ_MODE=12)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for i in 1 2 3; do for v in 0 12; do
  HPNN_FZ_MODE=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 2>&1 | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/mode=$v /" || exit 1
done; done
