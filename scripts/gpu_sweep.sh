#!/bin/bash
# Sweep of the fused-path knobs on one GPU: side-stream reduction, wide/narrow optimizer,
# split-K factor of the G0 GEMM.  Each bench runs under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${SWEEP_CFGS:-"0 0 0" "1 0 0" "0 1 0" "0 0 48" "0 1 48" "0 0 64" "0 1 64" "0 0 32" "0 1 40"}; do
  set -- $cfg
  log=gpurun_out/sw_side$1_narrow$2_s$3.log
  HPNN_SIDE_REDUCE=$1 HPNN_UPD_NARROW=$2 HPNN_TN_SPLITS=$3 timeout -k 10 120 python bench.py --steps ${STEPS:-400} --warmup 20 > $log 2>&1
  rc=$?
  echo "side=$1 narrow=$2 splits=$3 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $log)"
  [ $rc -eq 0 ] || exit $rc
done
