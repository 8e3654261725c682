#!/bin/bash
# A/B of the optimizer-update kernels (HPNN_UPD_MODE 0 = 8-row sub-tiles, 1 = 32x32 tiles):
# full GPU tests, then bench and a rocprofv3 kernel table for each mode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
for m in 1 0 1 0; do
  HPNN_UPD_MODE=$m timeout -k 10 120 python bench.py --steps 400 --warmup 20 > gpurun_out/ab_bench_$m.log 2>&1 || exit 1
  echo "mode=$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bench_$m.log)"
done
export TMPDIR=/tmp
for m in 1 0; do
  HPNN_UPD_MODE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_prof$m -o run -- python3 bench.py --steps 50 --warmup 10 --graph 0 > gpurun_out/ab_prof$m.log 2>&1 || exit 1
done
echo DONE
