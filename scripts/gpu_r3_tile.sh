set -e
for d in 3 5 7; do HPNN_TILE_D=$d timeout -k 10 120 python scripts/tile_bench.py --modes t > gpurun_out/tile_d$d.log 2>&1; done
timeout -k 10 700 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_tile_gpu.py tests/test_xar_gpu.py tests/test_fp_gpu.py tests/test_dp_xar_gpu.py > gpurun_out/t3.log 2>&1
