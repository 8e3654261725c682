#!/bin/bash
# RRUFF step: split-K row count of the non-8-phase weight gradients (HPNN_TN_ROWS -> G1's
# split count: 512 rows = 32 splits, the default), same box, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/rows; mkdir -p $O
for r in 512 256 1024 2048 512 256 1024; do
  HPNN_TN_ROWS=$r timeout -k 10 200 python bench.py --model rruff --steps 200 --warmup 20 > $O/r_$r.log 2>&1 || exit $?
  echo "rows=$r us=$(tail -n 1 $O/r_$r.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*1000)')"
done
