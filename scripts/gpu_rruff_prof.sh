#!/bin/bash
# RRUFF-shaped 4096-230-230 SNN and synthetic 8x4096 ANN steps: throughput, then per-kernel
# times under rocprofv3 (kernel trace + stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in rruff_snn synth_ann; do
  timeout -k 10 200 python scripts/bench_configs.py --only $c 2>&1 | grep '{' | tee -a gpurun_out/cfg_bench.txt || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o run -- python3 scripts/bench_configs.py --only $c --steps 20 > gpurun_out/prof_$c.log 2>&1 || { tail -20 gpurun_out/prof_$c.log; exit 1; }
  cut -d, -f1-4 gpurun_out/prof_$c/run_kernel_stats.csv | head -12
done
