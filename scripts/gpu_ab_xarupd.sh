#!/bin/bash
# A/B of the N > 1 MNIST step path on one GPU (HPNN_DP_FORCE=1): optimizer step fused into
# the xGMI all-reduce (HPNN_XAR_UPD=1) vs a separate update launch (0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export HPNN_DP_FORCE=1
R="-m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533"
for i in 1 2 3; do for v in 1 0; do
  HPNN_XAR_UPD=$v timeout -k 10 200 python $R bench.py --steps 400 --warmup 40 2>&1 | grep -o '"ms_per_step": [0-9.]*' | sed "s/^/upd=$v /" || exit 1
done; done
