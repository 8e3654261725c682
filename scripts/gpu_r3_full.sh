#!/bin/bash
# round 3: full GPU suite + tile timeline + bench, each step under its own limit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
HPNN_TILE_TRACE=1 timeout -k 10 120 python scripts/tile_trace.py > gpurun_out/trace1.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/full.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.log 2>&1
