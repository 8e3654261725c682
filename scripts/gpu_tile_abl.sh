#!/bin/bash
# tile front ablations (HPNN_TILE_ABL, profiling only): step time with half the W0 loads / no X loads
# needs a library built with `make ABLATIONS=1` (the default build ignores the variable)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab; mkdir -p $O
for v in 0 3 4 5 2 0; do
  HPNN_TILE_ABL=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 > $O/abl_$v.log 2>&1 || exit $?
  echo "abl=$v $(tail -n 1 $O/abl_$v.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*1000)')"
done
