#!/bin/bash
# round 4, call A: baseline bench (headline + rruff) and the FP64 online engine on a wide net
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/bench_mnist.json 2> $O/bench_mnist.err || { tail -20 $O/bench_mnist.err; exit 1; }
cat $O/bench_mnist.json
timeout -k 10 300 python bench.py --model rruff --steps 100 --warmup 10 > $O/bench_rruff.json 2> $O/bench_rruff.err || { tail -20 $O/bench_rruff.err; exit 1; }
cat $O/bench_rruff.json
bash scripts/gpu_online_wide.sh
