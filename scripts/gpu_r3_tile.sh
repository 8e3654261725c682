#!/bin/bash
# tile front: timeline + timing + its tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
HPNN_TILE_TRACE=1 timeout -k 10 120 python scripts/tile_trace.py > gpurun_out/trace2.log 2>&1 || exit $?
timeout -k 10 150 python scripts/tile_bench.py --modes t > gpurun_out/tile_b2.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_tile_gpu.py tests/test_g0_fm_gpu.py tests/test_model_gpu.py > gpurun_out/t4.log 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rruff -o run -- python3 bench.py --model rruff --steps 30 --warmup 5 --graph 0 > gpurun_out/prof_rruff.log 2>&1
