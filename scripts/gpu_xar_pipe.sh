#!/bin/bash
# xGMI all-reduce copy-in, 8 vs 16 slab loads in flight per thread (HPNN_XAR_U16): xar / DP
# tests, then the N = 1 step and the N > 1 step path (HPNN_DP_FORCE=1) alternating on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
HPNN_XAR_U16=1 timeout -k 10 300 python -u -m pytest tests/test_xar_gpu.py tests/test_dp_xar_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xarpipe_tests.log 2>&1 || { tail -30 gpurun_out/xarpipe_tests.log; exit 1; }
tail -2 gpurun_out/xarpipe_tests.log
R="-m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551"
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 400 --warmup 40 2>&1 | grep metric | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("N=1          ", round(d["ms_per_step"]*1e3,2), "us")' | tee -a gpurun_out/xar_u16.txt || exit 1
  for u in 0 1; do
    HPNN_XAR_U16=$u HPNN_DP_FORCE=1 timeout -k 10 200 python $R bench.py --steps 400 --warmup 40 2>&1 | grep metric | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("N>1 path u16='$u'", round(d["ms_per_step"]*1e3,2), "us")' | tee -a gpurun_out/xar_u16.txt || exit 1
  done
done
