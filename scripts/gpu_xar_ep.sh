#!/bin/bash
# xGMI all-reduce with cached-memory epochs: xar / DP tests, then the N = 1 step and the
# N > 1 step path (HPNN_DP_FORCE=1) alternating on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_xar_gpu.py tests/test_dp_xar_gpu.py tests/test_dp_mp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xarep_tests.log 2>&1 || { tail -30 gpurun_out/xarep_tests.log; exit 1; }
tail -2 gpurun_out/xarep_tests.log
R="-m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29553"
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 400 --warmup 40 2>&1 | grep metric | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("N=1     ", round(d["ms_per_step"]*1e3,2), "us")' | tee -a gpurun_out/xar_ep.txt || exit 1
  HPNN_DP_FORCE=1 timeout -k 10 200 python $R bench.py --steps 400 --warmup 40 2>&1 | grep metric | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("N>1 path", round(d["ms_per_step"]*1e3,2), "us")' | tee -a gpurun_out/xar_ep.txt || exit 1
done
