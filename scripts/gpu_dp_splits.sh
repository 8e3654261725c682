#!/bin/bash
# N > 1 MNIST step path on ONE GPU (HPNN_DP_FORCE=1) vs the first-layer gradient split count.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export HPNN_DP_FORCE=1
R="-m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29537"
for rep in 1 2; do
  for s in 32 40 48 64; do
    out=$(HPNN_TN_SPLITS=$s timeout -k 10 200 python $R bench.py --steps 400 --warmup 40 2>&1 | grep metric) || exit 1
    echo "splits=$s $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,2), "us", d["config"]["grad_allreduce"])')" | tee -a gpurun_out/dp_splits.txt
  done
done
