#!/bin/bash
# One GPU call = a list of named steps, each under its own time limit; a crash / fault / timeout
# (rc not 0 or 1) ends the call.  Output: gpurun_out/<tag>/<step>.log, steps.log.
#
#   usage: scripts/gpu.sh <tag> <step>[+VAR=VAL...] [<step>[+VAR=VAL...] ...]
#
# A step may carry environment settings after "+" (e.g. bench+HPNN_TILE_PP=4); each step's
# log name starts with the step's position.  Steps:
#   tests                 the whole GPU suite            tests:<expr>  pytest -m gpu -k <expr>
#   smoke                 __graft_entry__.smoke()        bench         MNIST headline (200 steps)
#   rruff / synth / synth1k   bench.py --model rruff | synth | synth at batch 1024
#   dpforce               the N > 1 MNIST path with one rank under torchrun
#   dpforce_synth1k[_bf16]  the same for synth at batch 1024 (FP32 exchange / the BF16 reduce-scatter path)
#   dpemu8_synth1k / prof_dpemu8   one rank running the sharded step at 8-rank sizes (HPNN_DPX_EMULATE_WORLD=8)
#   trace                 tile-front phase trace (HPNN_TILE_TRACE=1)
#   prof / prof_rruff     rocprofv3 kernel table (--graph 0)
#   pmc / pmc_rruff       PMC passes of the step (scripts/pmc_step.sh); pmc_d8: 8 cycled batches
#   rehearse              2 ranks sharing the GPU (scripts/rehearse.sh)
#   libbench / libbench_dp   train_nn vs bench.py (scripts/lib_vs_bench.py; _dp: the N > 1 path, one rank)
#   learn                 scripts/learnability.py
#   cache                 headline with 4 vs 8 cycled batches (Infinity-Cache sensitivity)
#   py:<script args>      python scripts/<script> <args> (spaces as ',')
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
O=gpurun_out/$tag; mkdir -p $O
step() {  # step <name> <timeout> <cmd...>   (log: <NN>_<name>.log, NN = position on the command line)
  local name=$(printf "%02d" $IDX)_$1 t=$2; shift 2
  echo "=== $name [$STEP_ENV]: $*" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $O/steps.log
  tail -n 12 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  [ $rc -eq 1 ] && FAILED=1
  return 0
}
export TMPDIR=/tmp
FAILED=0
port=29600
IDX=0
for spec in "$@"; do
  IDX=$((IDX + 1))
  s=${spec%%+*}
  envs=()
  STEP_ENV=""
  if [ "$spec" != "$s" ]; then IFS='+' read -ra envs <<< "${spec#*+}"; STEP_ENV="${spec#*+}"; fi
  port=$((port + 1))
  (
  for e in "${envs[@]}"; do export "$e"; done
  case $s in
    tests) step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    tests:*) step pytest_sel 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${s#tests:}" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 300 python bench.py --steps 200 --warmup 20 ;;
    rruff) step bench_rruff 300 python bench.py --model rruff --steps 100 --warmup 10 ;;
    synth) step bench_synth 300 python bench.py --model synth --steps 20 --warmup 5 ;;
    synth1k) step bench_synth1k 300 python bench.py --model synth --batch 1024 --steps 50 --warmup 10 ;;
    dpforce) HPNN_DP_FORCE=1 step dpforce 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --steps 200 --warmup 20 ;;
    dpforce_synth1k) HPNN_DP_FORCE=1 step dpforce_synth1k 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --model synth --batch 1024 --steps 50 --warmup 10 ;;
    dpforce_synth1k_bf16) HPNN_DP_FORCE=1 HPNN_DPX_FORCE=1 HPNN_DPX_SHARD1=1 step dpforce_synth1k_bf16 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --model synth --batch 1024 --steps 50 --warmup 10 --grad-comm bf16rs ;;
    dpemu8_synth1k) HPNN_DP_FORCE=1 HPNN_DPX_FORCE=1 HPNN_DPX_EMULATE_WORLD=8 step dpemu8_synth1k 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --model synth --batch 1024 --steps 50 --warmup 10 --grad-comm bf16rs ;;
    prof_dpemu8) HPNN_DP_FORCE=1 HPNN_DPX_FORCE=1 HPNN_DPX_EMULATE_WORLD=8 step rocprof_dpemu8 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dpemu8 -o run -- python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --model synth --batch 1024 --steps 20 --warmup 5 --graph 0 --grad-comm bf16rs ;;
    trace) HPNN_TILE_TRACE=1 step tile_trace 200 python scripts/tile_trace.py ;;
    trace1) HPNN_TILE_TRACE=1 step tile_trace_d1 200 python scripts/tile_trace.py 1 ;;
    g0trace) HPNN_G0_TRACE=1 step g0_trace 200 python scripts/g0_trace.py ;;
    prof) step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 50 --warmup 10 --graph 0 ;;
    prof_rruff) step rocprof_rruff 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rruff -o run -- python3 bench.py --model rruff --steps 30 --warmup 5 --graph 0 ;;
    prof_synth1k_noupd) HPNN_TN_UPD=0 step rocprof_synth1k_noupd 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_synth1k_noupd -o run -- python3 bench.py --model synth --batch 1024 --steps 20 --warmup 5 --graph 0 ;;
    prof_synth1k) step rocprof_synth1k 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_synth1k -o run -- python3 bench.py --model synth --batch 1024 --steps 20 --warmup 5 --graph 0 ;;
    pmc) PMC_TAG=_$tag step pmc 600 bash scripts/pmc_step.sh ;;
    pmc_rruff) PMC_TAG=_${tag}_rruff step pmc_rruff 600 bash scripts/pmc_step.sh --model rruff ;;
    pmc_d8) PMC_TAG=_${tag}_d8 step pmc_d8 600 bash scripts/pmc_step.sh --datasets 8 ;;
    rehearse) step rehearse 600 bash scripts/gpu_rehearse.sh ;;
    libbench) step libbench 900 python scripts/lib_vs_bench.py --out $O/lib_vs_bench.jsonl ;;
    libbench_dp) step libbench_dp 900 python scripts/lib_vs_bench.py --dpforce --configs mnist --out $O/lib_vs_bench_dp.jsonl ;;
    learn) step learn 600 python scripts/learnability.py --out $O/learnability.jsonl ;;
    cache) step cache_d1 300 python bench.py --steps 200 --warmup 20 --datasets 1 &&
           step cache_d4 300 python bench.py --steps 200 --warmup 20 --datasets 4 &&
           step cache_d8 300 python bench.py --steps 200 --warmup 20 --datasets 8 &&
           step cache_d4b 300 python bench.py --steps 200 --warmup 20 --datasets 4 &&
           step cache_d8b 300 python bench.py --steps 200 --warmup 20 --datasets 8 ;;
    py:*) a=${s#py:}; step "py_$(basename ${a%%,*} .py)" 600 python scripts/${a//,/ } ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  exit $FAILED
  )
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
