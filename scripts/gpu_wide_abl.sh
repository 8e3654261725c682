#!/bin/bash
# wide front ablations (HPNN_WIDE_ABL): whole kernel, phase A alone, everything but phase A
# needs a library built with `make ABLATIONS=1` (the default build ignores the variable)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/wide; mkdir -p $O
for v in 0 1 2 3 4 5; do
  HPNN_WIDE_ABL=$v timeout -k 10 120 python scripts/wide_bench.py --iters 100 > $O/abl_$v.log 2>&1 || exit $?
  echo "abl=$v $(grep wide2_front $O/abl_$v.log)"
done
