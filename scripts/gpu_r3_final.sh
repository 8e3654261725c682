#!/bin/bash
# round 3 end-of-session validation: GPU suite, smoke, the three bench configs, kernel tables,
# PMC memory-side bytes of the MNIST step, tile phase timeline.  Each GPU step has its own
# limit; a failing step ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final; mkdir -p $O; export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; tail -n 3 $O/gputest.log; if [ $rc -ne 0 ]; then exit $rc; fi
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -n 1 $O/smoke.log
for m in mnist mnist rruff synth; do
  st=200; [ $m = synth ] && st=20
  $T 300 python bench.py --model $m --steps $st --warmup 10 > $O/bench_$m.log 2>&1 || exit $?
  tail -n 1 $O/bench_$m.log >> $O/bench.jsonl
done
$T 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mnist -o p -- python3 bench.py --steps 50 --warmup 10 --graph 0 > $O/prof_mnist.log 2>&1 || exit $?
$T 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rruff -o p -- python3 bench.py --model rruff --steps 50 --warmup 10 --graph 0 > $O/prof_rruff.log 2>&1 || exit $?
PMC_TAG=_final bash scripts/pmc_step.sh > $O/pmc.log 2>&1 || exit $?
HPNN_TILE_TRACE=1 $T 120 python scripts/tile_trace.py > $O/tile_trace.log 2>&1 || exit $?
echo done
