#!/bin/bash
# Front-kernel iteration: fused-path tests on the role-split kernel, per-kernel times for
# both front kernels (default mlp3_fused, HPNN_FRONT=f mlp3_front) and its ablation modes
# (HPNN_FZ_MODE), the timeline, and the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n ${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
HPNN_FRONT=f step tests 600 python -u -m pytest tests/test_model_gpu.py tests/test_racecheck_gpu.py -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
TAILN=3 step kb_x 200 python scripts/kbench.py --modes x --reps 10
HPNN_FRONT=f TAILN=3 step kb_f 200 python scripts/kbench.py --modes x --reps 10
for m in ${MODES:-1 2 3}; do HPNN_FRONT=f HPNN_FZ_MODE=$m TAILN=3 step kb_m$m 200 python scripts/kbench.py --modes x --reps 10; done
HPNN_FRONT=f HPNN_FZ_MODE=9 TAILN=14 step trace 200 python scripts/fz_trace.py
HPNN_FRONT=f step bench 300 python bench.py --steps 200 --warmup 20
echo DONE
