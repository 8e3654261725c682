#!/bin/bash
# One gpurun call: GPU tests, smoke, bench, rocprof summary.  Every GPU step has its own
# time limit; a crash/fault/timeout (rc not in {0,1}) stops the script immediately.
# usage: scripts/gpu_round.sh [tests|bench|prof|all] [extra pytest args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
what=${1:-all}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ "$what" = tests ] || [ "$what" = all ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${@:2}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  step bench 300 python bench.py --steps 200 --warmup 20
fi
if [ "$what" = prof ] || [ "$what" = all ]; then
  export TMPDIR=/tmp
  step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 10 --graph 0
fi
echo DONE
