#!/bin/bash
# DP path on one GPU: single-rank RCCL process group (HPNN_DP_FORCE=1), eager and graph-captured.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 180 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dp_test.log 2>&1 || { tail -30 gpurun_out/dp_test.log; exit 1; }
tail -3 gpurun_out/dp_test.log
export HPNN_DP_FORCE=1
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 100 --warmup 10 > gpurun_out/dp_eager.log 2>&1 || { tail -30 gpurun_out/dp_eager.log; exit 1; }
tail -1 gpurun_out/dp_eager.log
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 1 --steps 100 --warmup 10 --graph 2 > gpurun_out/dp_graph.log 2>&1 || { tail -30 gpurun_out/dp_graph.log; exit 1; }
tail -1 gpurun_out/dp_graph.log
