#!/bin/bash
# device-spanning online engine (loopback slots) + wide FP64 online it/s + tile timeline/timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_capi_gpu.py -k "online" > gpurun_out/online_t.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/online_bench.py --dims 4096,4096,230 --n 5 --env '' --env HPNN_ONLINE_SLOTS=2 --out gpurun_out/online_wide.json > gpurun_out/online_b.log 2>&1 || exit $?
HPNN_TILE_TRACE=1 timeout -k 10 120 python scripts/tile_trace.py > gpurun_out/trace3.log 2>&1 || exit $?
timeout -k 10 150 python scripts/tile_bench.py --modes t > gpurun_out/tile_b3.log 2>&1 || exit $?
timeout -k 10 200 python bench.py > gpurun_out/bench1.log 2>&1
