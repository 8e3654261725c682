#!/bin/bash
# alternating bench A/B of the first-layer gradient kernel: default (LDS-DMA TN) vs HPNN_G0_RS=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for i in 1 2 3; do
  for v in 0 1; do
    HPNN_G0_RS=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 2>&1 | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/rs=$v /" || exit 1
  done
done
