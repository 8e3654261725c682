#!/bin/bash
# FP64 online engine (reference semantics) on a wide net: one device, two virtual slots,
# and train_nn -S 2 (two stream slots); then the MNIST tutorial shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/online; mkdir -p $O
timeout -k 10 400 python scripts/online_bench.py --dims 4096,4096,230 --n 6 --env '' --env HPNN_ONLINE_SLOTS=2 --env=-S2 --out $O/wide.json > $O/wide.log 2>&1 || { tail -20 $O/wide.log; exit 1; }
cat $O/wide.log
timeout -k 10 200 python scripts/online_bench.py --dims 784,300,10 --n 20 --train BP --net ANN --env '' --env=-S2 --out $O/mnist.json > $O/mnist.log 2>&1 || { tail -20 $O/mnist.log; exit 1; }
cat $O/mnist.log
