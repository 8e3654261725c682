#!/bin/bash
# A/B of the two MLP front kernels in the full MNIST step (bench.py, HIP graph), alternating
# runs on one box: default mlp3_fused vs HPNN_FRONT=f mlp3_front.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for f in x f; do
    HPNN_FRONT=$f timeout -k 10 120 python bench.py --steps 400 --warmup 40 > gpurun_out/ab_$f$i.log 2>&1 || exit $?
    echo "front=$f run $i: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$f$i.log)"
  done
done
