#!/bin/bash
# same-box A/B of two libhpnn builds: build_ab/libhpnn.so (A, via LD_LIBRARY_PATH: the Python
# module's RUNPATH yields to it) vs the in-tree build (B); usage: gpu_lib_ab.sh [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/libab; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_tile_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -n 1 $O/t.log
for r in 1 2 3; do
  LD_LIBRARY_PATH=$PWD/build_ab:$LD_LIBRARY_PATH $T 200 python bench.py --steps 300 --warmup 30 "$@" > $O/a_$r.log 2>&1 || exit $?
  $T 200 python bench.py --steps 300 --warmup 30 "$@" > $O/b_$r.log 2>&1 || exit $?
  echo "A $(tail -n 1 $O/a_$r.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*1000)')  B $(tail -n 1 $O/b_$r.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*1000)')"
done
LD_LIBRARY_PATH=$PWD/build_ab:$LD_LIBRARY_PATH HPNN_TILE_TRACE=1 $T 120 python scripts/tile_trace.py > $O/trA.log 2>&1 || exit $?
HPNN_TILE_TRACE=1 $T 120 python scripts/tile_trace.py > $O/trB.log 2>&1 || exit $?
paste <(grep ticks $O/trA.log | cut -c1-60) <(grep ticks $O/trB.log | cut -c29-60)
