#!/bin/bash
# tile front: numerics tests, repeated bench step times (one box), phase timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_tile_gpu.py tests/test_g0_fm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t8.log 2>&1 || exit $?
for v in 1 2 3; do
  $T 200 python bench.py --steps 300 --warmup 30 > $O/b_$v.log 2>&1 || exit $?
  echo "run $v $(tail -n 1 $O/b_$v.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*1000)')"
done
HPNN_TILE_TRACE=1 $T 120 python scripts/tile_trace.py > $O/tr8.log 2>&1 || exit $?
grep -v amdgpu.ids $O/tr8.log
