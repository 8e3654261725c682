#!/bin/bash
# round 3: GPU suite, the three bench configs, a rocprofv3 kernel table of the headline
# bench and one PMC pass (DRAM bytes) -- each GPU step under its own limit, chained so a
# fault ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
O=gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; tail -3 $O/gputest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 200 --warmup 20 > $O/bench_mnist.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --model rruff --steps 100 --warmup 10 > $O/bench_rruff.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --model synth --steps 20 --warmup 5 > $O/bench_synth.log 2>&1 || exit $?
tail -1 $O/bench_mnist.log $O/bench_rruff.log $O/bench_synth.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mnist -o p -- python3 bench.py --steps 50 --warmup 10 --graph 0 > $O/prof_mnist.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rruff -o p -- python3 bench.py --model rruff --steps 50 --warmup 10 --graph 0 > $O/prof_rruff.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_mnist -o p -- python3 bench.py --steps 20 --warmup 5 --graph 0 > $O/pmc_mnist.log 2>&1
echo "pmc rc=$?"
