#!/bin/bash
# MNIST step: split-K count of the first-layer gradient G0 (HPNN_TN_SPLITS; only G0 is a
# separate GEMM in the tile-front step, 48 = the default), same box, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/g0s; mkdir -p $O
for r in 48 32 40 56 64 24 48 32 40 56 64; do
  HPNN_TN_SPLITS=$r timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/s_$r.log 2>&1 || exit $?
  echo "splits=$r us=$(tail -n 1 $O/s_$r.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*1000)')"
done
