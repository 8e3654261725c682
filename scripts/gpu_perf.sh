#!/bin/bash
# Perf iteration on one GPU: kernel tests, bench, split-K sweep of the G0 GEMM, rocprof stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local n=$1 t=$2; shift 2; echo "=== $n: $*"; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; tail -n ${TAILN:-3} "gpurun_out/$n.log"; echo "=== $n rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo ABORT; exit $rc; fi; [ $rc -eq 0 ] || exit 1; }
TAILN=4 run kt 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_dp_gpu.py -x -q --timeout 120 --timeout-method thread
run bench 200 python bench.py --steps 200 --warmup 20
for S in ${SWEEP:-48 64 96 128}; do HPNN_TN_SPLITS=$S run bench_s$S 200 python bench.py --steps 200 --warmup 20; done
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 10 --graph 0
python3 scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv gpurun_out/trace_summary.md
echo DONE
