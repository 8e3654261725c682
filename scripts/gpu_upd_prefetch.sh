#!/bin/bash
# MNIST step with the update kernel fetching W / V before its slab sum: tests of the update,
# then bench.py (3 runs) and the N > 1 path on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_racecheck_gpu.py -x -q -k "sgd or update or train_step or deterministic or fused" --timeout 120 --timeout-method thread > gpurun_out/upd_tests.log 2>&1 || { tail -30 gpurun_out/upd_tests.log; exit 1; }
tail -2 gpurun_out/upd_tests.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 400 --warmup 40 2>&1 | grep metric | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("N=1", round(d["ms_per_step"]*1e3,2), "us")' | tee -a gpurun_out/upd_prefetch.txt || exit 1
done
