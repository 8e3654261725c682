#!/bin/bash
# The N > 1 data-parallel step path (xGMI all-reduce with slab sums in its copy-in) timed on
# ONE GPU: torchrun with one rank and HPNN_DP_FORCE=1; then a rocprofv3 kernel trace of it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
export HPNN_DP_FORCE=1
R="-m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531"
timeout -k 10 200 python bench.py --steps 200 --warmup 20 2>&1 | grep metric || exit 1
timeout -k 10 200 python $R bench.py --steps 200 --warmup 20 2>&1 | grep metric || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dpf -o run -- python3 $R bench.py --steps 30 --warmup 5 --graph 0 > gpurun_out/dpf.log 2>&1 || exit 1
cut -d, -f1-4 gpurun_out/dpf/run_kernel_stats.csv | head -12
