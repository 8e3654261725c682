#!/bin/bash
# bench.py --model for the other BASELINE configs: one GPU, and the N > 1 (data-parallel)
# step path on one GPU (HPNN_DP_FORCE=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
R="-m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541"
timeout -k 10 200 python bench.py --steps 40 --warmup 5 2>&1 | grep metric | tee -a gpurun_out/bench_models.txt || exit 1
for m in rruff synth; do
  st=200; [ $m = synth ] && st=20
  timeout -k 10 300 python bench.py --model $m --steps $st --warmup 5 2>&1 | grep metric | tee -a gpurun_out/bench_models.txt || exit 1
  HPNN_DP_FORCE=1 timeout -k 10 300 python $R bench.py --model $m --steps $st --warmup 5 2>&1 | grep metric | tee -a gpurun_out/bench_models.txt || exit 1
done
