#!/bin/bash
# round 3: GPU suite (all failures, not just the first) + phase timelines of the tile
# front (MNIST) and the wide front (RRUFF)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3; mkdir -p $O
export TMPDIR=/tmp
HPNN_TILE_TRACE=1 timeout -k 10 120 python scripts/tile_trace.py > $O/tile_trace.log 2>&1 || exit $?
HPNN_WIDE_TRACE=1 timeout -k 10 120 python scripts/wide_bench.py > $O/wide_trace.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 150 --timeout-method thread > $O/gputest2.log 2>&1
rc=$?; tail -n 15 $O/gputest2.log; exit $rc
