#!/bin/bash
# xGMI all-reduce launch shape on the N > 1 MNIST step path, timed on ONE GPU
# (HPNN_DP_FORCE=1: one rank, the all-reduce with its 48-slab copy-in and fused update
# still runs): workgroups (threads per workgroup were swept too: 512 / 1024 slower, the
# knob is gone), alternating order, plus the xar tests
# (attach-time self-test included).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_xar_gpu.py tests/test_dp_xar_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xar_tests.log 2>&1 || { tail -30 gpurun_out/xar_tests.log; exit 1; }
tail -2 gpurun_out/xar_tests.log
export HPNN_DP_FORCE=1
R="-m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533"
for rep in 1 2; do
  for cfg in "128 256" "256 256"; do
    set -- $cfg
    out=$(HPNN_XAR_BLOCKS=$1 timeout -k 10 200 python $R bench.py --steps 400 --warmup 40 2>&1 | grep metric) || exit 1
    echo "blocks=$1 threads=$2 $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,2), "us", d["config"]["grad_allreduce"])')" | tee -a gpurun_out/xar_grid.txt
  done
done
