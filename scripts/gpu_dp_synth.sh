#!/bin/bash
# data-parallel tests, then the synthetic config's N > 1 step path on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dp_gpu.py tests/test_dp_xar_gpu.py tests/test_dp_mp_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dp_tests.log 2>&1 || { tail -30 gpurun_out/dp_tests.log; exit 1; }
tail -2 gpurun_out/dp_tests.log
R="-m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29543"
for m in synth rruff; do
  st=200; [ $m = synth ] && st=20
  HPNN_DP_FORCE=1 timeout -k 10 300 python $R bench.py --model $m --steps $st --warmup 5 2>&1 | grep metric | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["metric"][:60], round(d["ms_per_step"],4), "ms")' | tee -a gpurun_out/dp_synth.txt || exit 1
done
