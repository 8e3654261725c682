set -o pipefail
mkdir -p gpurun_out/ab
HPNN_TN_DEEP=1 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_deep.log 2>&1 || exit 1
for cfg in "0 48" "1 48" "0 48" "1 48" "1 32" "1 40" "1 64" "1 96"; do
  set -- $cfg
  HPNN_TN_DEEP=$1 HPNN_TN_SPLITS=$2 timeout -k 10 120 python bench.py --steps 400 > gpurun_out/ab/b_$1_$2.log 2>&1 || exit 1
  echo "deep=$1 splits=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/b_$1_$2.log)" | tee -a gpurun_out/ab/summary.txt
done
