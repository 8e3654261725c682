#!/bin/bash
# wide-input front: tests + kernel table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread tests/test_wide_gpu.py > gpurun_out/wide_t.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rruff2 -o run -- python3 bench.py --model rruff --steps 30 --warmup 5 --graph 0 > gpurun_out/prof_rruff2.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --model rruff --steps 30 --warmup 5 > gpurun_out/bench_rruff2.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_capi_gpu.py -k "device_spanning or tensor_parallel" > gpurun_out/online_t2.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/online_bench.py --dims 4096,4096,230 --n 5 --env '' --env HPNN_ONLINE_SLOTS=2 --out gpurun_out/online_wide.json > gpurun_out/online_b.log 2>&1
