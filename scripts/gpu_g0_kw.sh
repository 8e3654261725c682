#!/bin/bash
# G0 (MNIST first-layer gradient): 2 vs 3 k-interleaved wave groups per workgroup
# (HPNN_G0_KW), numerics with 3 groups first, then the step time interleaved on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/g0kw; mkdir -p $O
HPNN_G0_KW=3 timeout -k 10 300 python -u -m pytest tests/test_g0_fm_gpu.py tests/test_tile_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -n 1 $O/t.log
for k in 2 3 2 3 2 3; do
  HPNN_G0_KW=$k timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/k_$k.log 2>&1 || exit $?
  echo "kw=$k us=$(tail -n 1 $O/k_$k.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"]*1000)')"
done
export TMPDIR=/tmp
for k in 2 3; do
  HPNN_G0_KW=$k timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$k -o p -- python3 bench.py --steps 50 --warmup 10 --graph 0 > $O/prof_$k.log 2>&1 || exit $?
  python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof_$k/p_kernel_stats.csv')))[:4]: print('kw=$k', r['Name'][:40], round(float(r['AverageNs'])/1e3,2))"
done
