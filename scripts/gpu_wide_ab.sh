#!/bin/bash
# wide (RRUFF) front: numerics tests, ablations, bench step time, kernel table
# needs a library built with `make ABLATIONS=1` (the default build ignores the variable)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/wide; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_wide_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -n 1 $O/t.log
for v in 0 1 2 3; do
  HPNN_WIDE_ABL=$v $T 120 python scripts/wide_bench.py --iters 100 > $O/abl_$v.log 2>&1 || exit $?
  echo "abl=$v $(grep wide2_front $O/abl_$v.log)"
done
$T 200 python bench.py --model rruff --steps 100 --warmup 10 > $O/b.log 2>&1 || exit $?
echo "rruff step us: $(tail -n 1 $O/b.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*1000)')"
$T 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --model rruff --steps 30 --warmup 5 --graph 0 > $O/prof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open("gpurun_out/wide/prof/p_kernel_stats.csv")))
for r in rows[:6]:
    print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:8.2f}")
PY
