#!/bin/bash
# bench A/B: 8-bit pixel input (fragment-major 8-bit G0 operand) vs float input (TN G0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for i in 1 2 3; do for v in u8 float; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 --input $v 2>&1 | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/$v /" || exit 1
done; done
