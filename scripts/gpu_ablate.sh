#!/bin/bash
# Read-bandwidth probe + mlp3_fused ablation modes (HPNN_FZ_MODE) + per-kernel times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 bench_micro/stream_read > gpurun_out/stream_read.log 2>&1 || exit $?
cat gpurun_out/stream_read.log
for m in 0 1 2 3 4 5 6 7 8 10; do
  HPNN_FZ_MODE=$m timeout -k 10 120 python scripts/kbench.py --modes x --reps 10 > gpurun_out/ablate_$m.log 2>&1 || exit $?
  echo "mode $m: $(grep -E 'fused front|grad_l0|full' gpurun_out/ablate_$m.log | tr -s ' ' | tr '\n' '|')"
done
