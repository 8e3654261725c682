#!/bin/bash
# xGMI all-reduce: GPU tests, then per-call protocol cost (scripts/xar_bench.py) per mode /
# world / fence variant, all ranks on the box's one GPU.  usage: scripts/gpu_xar.sh [notest]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
if [ "$1" != notest ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_xar_gpu.py tests/test_dp_xar_gpu.py > gpurun_out/xar_tests.log 2>&1
  rc=$?; tail -12 gpurun_out/xar_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for f in 1 0; do for w in 1 2 4; do for m in 1 2; do
  HPNN_XAR_FENCE=$f timeout -k 10 120 python scripts/xar_bench.py --world $w --mode $m 2>&1 | grep world | sed "s/^/fence=$f /" || exit $?
done; done; done
