#!/bin/bash
# Rehearsal of the driver's N > 1 bench path on ONE GPU: torchrun with 2 ranks sharing the
# card (HPNN_BENCH_REHEARSE=1: gloo group, xGMI all-reduce kernel only, HIP graphs).  Not 4:
# three ranks' spinning all-reduce workgroups can then hold every CU the fourth rank's
# persistent front kernel needs, the barrier times out (bounded, 5 s) and the run falls back
# to torch.distributed -- an artefact of ranks sharing one card (the 4-rank protocol itself
# is covered by tests/test_xar_gpu.py with small kernels).
# Checks that every rank runs, the all-reduce self-test and barriers pass, rank 0 prints
# one JSON line; the per-step time of ranks sharing one GPU is not a scaling number.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export HPNN_BENCH_REHEARSE=1
for n in 2; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 40 --warmup 5 > gpurun_out/rehearse_$n.log 2>&1 || { tail -30 gpurun_out/rehearse_$n.log; exit 1; }
  grep -c '"metric"' gpurun_out/rehearse_$n.log
  grep '"metric"' gpurun_out/rehearse_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["n_gpus"], d["config"]["parallelism"], d["config"]["grad_allreduce"], d["config"]["hip_graph"], round(d["ms_per_step"]*1e3,1), "us/step (ranks sharing one GPU)")'
  grep -i "self-test\|timed out\|error" gpurun_out/rehearse_$n.log | head -5
done
# the driver's exact N > 1 MNIST path (exchange inside the G0 launch, HIP graphs) with 2 ranks:
# per-rank batch 8192, so both ranks' G0 grids (80 workgroups each) and fronts fit at once
HPNN_REHEARSE_FUSED=1 HPNN_SPLITS=8,0,0 timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 40 --warmup 5 --batch 8192 > gpurun_out/rehearse_fused.log 2>&1 || { tail -30 gpurun_out/rehearse_fused.log; exit 1; }
grep '"metric"' gpurun_out/rehearse_fused.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("fused", d["n_gpus"], d["config"]["parallelism"], d["config"]["grad_allreduce"], d["config"].get("grad_exchange"), d["config"]["hip_graph"], round(d["ms_per_step"]*1e3,1), "us/step (ranks sharing one GPU, batch 8192 per rank)")'
grep -i "self-test\|timed out\|error" gpurun_out/rehearse_fused.log | head -5
