#!/bin/bash
# Development iteration on the GPU box: kernel tests, per-kernel microbench, short bench,
# kernel-trace profile of the graphed bench.  Each GPU step has its own time limit and a
# crash/fault/timeout stops the script.   usage: scripts/gpu_iter.sh [pytest-args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 30
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_k 600 python -m pytest ${PYTEST_FILES:-tests/test_kernels_gpu.py tests/test_model_gpu.py} -x -q ${PYTEST_ARGS:-}
step kbench 300 python scripts/kbench.py --reps 10
step bench 300 python bench.py --steps 200 --warmup 20
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 10
echo DONE
