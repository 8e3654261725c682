#!/bin/bash
# round-4 GPU call: steps by name, each under its own time limit; a crash / fault / timeout
# (rc not 0 or 1) ends the call.   usage: scripts/gpu_r4.sh <tag> <step> [<step> ...]
#   steps: tests | tests:<pytest -k expr> | smoke | bench | rruff | synth | synthrs | libbench | fpbench |
#          learn | prof | prof0 | prof_rruff | fpsteps | pmc | pmc_rruff | trace | rehearse | dpforce |
#          dpprof | A/B sets: mnistab rruffab rruffab2 earlyab dpab xchgab pfab xarb g0s rruffs t64ab
#          tradeab xordab gsab synthab tnr widetr
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
O=gpurun_out/$tag; mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $O/steps.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $O/steps.log
  tail -n 15 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
export TMPDIR=/tmp
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    tests:*) step pytest_sel 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${s#tests:}" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 300 python bench.py --steps 200 --warmup 20 ;;
    rruff) step bench_rruff 300 python bench.py --model rruff --steps 100 --warmup 10 ;;
    synth) step bench_synth 300 python bench.py --model synth --steps 20 --warmup 5 ;;
    libbench) step libbench 900 python scripts/lib_vs_bench.py --out $O/lib_vs_bench.jsonl ;;
    fpbench) step fpbench 300 python scripts/gemm_fp_bench.py --out $O/gemm_fp.jsonl ;;
    prof) step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 50 --warmup 10 --graph 0 ;;
    prof0) HPNN_G0_FUSED=0 step rocprof0 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof0 -o run -- python3 bench.py --steps 50 --warmup 10 --graph 0 ;;
    prof_rruff) step rocprof_rruff 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rruff -o run -- python3 bench.py --model rruff --steps 30 --warmup 5 --graph 0 ;;
    fpsteps) step fpsteps 600 python scripts/lib_vs_bench.py --dtype f64 --configs mnist,rruff,wide --batches 2 --epochs 3 --out $O/fp64_steps.jsonl ;;
    rruffab)  # G1 split variants on the fused 8-phase TN reduction + update
      step rruff_s32 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_SPLITS=16,64 HPNN_TN8_MINWG=64 step rruff_s64 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_SPLITS=16,128 step rruff_s128 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_SPLITS=16,64 step rruff_s64u 200 python bench.py --model rruff --steps 100 --warmup 10 ;;
    mnistab)  # fused G0 (2 launches) vs G0 + update launch, interleaved on one box
      step mnist_f1 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_G0_FUSED=0 step mnist_f0 200 python bench.py --steps 200 --warmup 20 &&
      step mnist_f1b 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_G0_FUSED=0 step mnist_f0b 200 python bench.py --steps 200 --warmup 20 ;;
    pmc) PMC_TAG=_$tag step pmc 600 bash scripts/pmc_step.sh ;;
    pmc_rruff) PMC_TAG=_${tag}_rruff step pmc_rruff 600 bash scripts/pmc_step.sh --model rruff ;;
    trace) HPNN_TILE_TRACE=1 step tile_trace 200 python scripts/tile_trace.py ;;
    rruffab2)  # fused 8-phase TN split-K reduction + step (layer 0) vs slabs + update launch
      step rruff_t1 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_TN8_FUSED=0 step rruff_t0 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      step rruff_t1b 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_TN8_FUSED=0 step rruff_t0b 200 python bench.py --model rruff --steps 100 --warmup 10 ;;
    dpforce)  # the N > 1 MNIST step path (xGMI all-reduce + update) timed with one rank on this GPU
      HPNN_DP_FORCE=1 step dpforce 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --steps 200 --warmup 20 ;;
    earlyab)  # tile front: X(s+2) conversion before (default) / after (HPNN_TILE_EARLY=0) the MFMAs
      step early1 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_TILE_EARLY=0 step early0 200 python bench.py --steps 200 --warmup 20 &&
      step early1b 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_TILE_EARLY=0 step early0b 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_TILE_TRACE=1 step trace1 200 python scripts/tile_trace.py &&
      HPNN_TILE_EARLY=0 HPNN_TILE_TRACE=1 step trace0 200 python scripts/tile_trace.py ;;
    dpprof)  # kernel table of the N > 1 MNIST step path, one process (env rendezvous, no launcher)
      HPNN_DP_FORCE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 step dpprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dpprof -o run -- python3 bench.py --steps 50 --warmup 10 --graph 0 &&
      HPNN_DP_FORCE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29534 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 step dpbench 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_XAR_UPD=0 HPNN_DP_FORCE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29535 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 step dpbench_sep 200 python bench.py --steps 200 --warmup 20 ;;
    dpab)  # N > 1 step path on one GPU: exchange inside the G0 launch vs its own launch (HPNN_XAR_G0=0), vs single
      step dpab_single 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_DP_FORCE=1 step dpab_local 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --steps 200 --warmup 20 &&
      HPNN_XAR_G0=0 HPNN_DP_FORCE=1 step dpab_buffer 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29542 bench.py --steps 200 --warmup 20 &&
      step dpab_singleb 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_DP_FORCE=1 step dpab_localb 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29543 bench.py --steps 200 --warmup 20 &&
      HPNN_XAR_G0=0 HPNN_DP_FORCE=1 step dpab_bufferb 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29544 bench.py --steps 200 --warmup 20 ;;
    xchgab)  # in-kernel exchange ablations (HPNN_G0_PROTO: 8 + system acquire, 16 no barrier)
      for pr in 0 8 16; do HPNN_G0_PROTO=$pr HPNN_DP_FORCE=1 step xchg_p$pr 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29550 + pr)) bench.py --steps 200 --warmup 20 || exit 1; done ;;
    xarb)  # all-reduce per-call protocol cost, 1 and 2 processes on this GPU
      step xarb_w1 200 python scripts/xar_bench.py --world 1 &&
      step xarb_w2 200 python scripts/xar_bench.py --world 2 &&
      step xarb_w2m2 200 python scripts/xar_bench.py --world 2 --mode 2 ;;
    pfab)  # fused G0: first stepped element's W / V prefetched after the GEMM (default) vs not (HPNN_G0_PROTO=64)
      step pf1 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_G0_PROTO=64 step pf0 200 python bench.py --steps 200 --warmup 20 &&
      step pf1b 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_G0_PROTO=64 step pf0b 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_DP_FORCE=1 step pfdp1 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --steps 200 --warmup 20 &&
      HPNN_G0_PROTO=64 HPNN_DP_FORCE=1 step pfdp0 200 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29562 bench.py --steps 200 --warmup 20 ;;
    rruffs)  # RRUFF G0 / G1 split sweep in the step
      step rs_def 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_SPLITS=8,32 step rs_8_32 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_SPLITS=32,32 step rs_32_32 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_SPLITS=16,16 step rs_16_16 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      step rs_defb 200 python bench.py --model rruff --steps 100 --warmup 10 ;;
    t64ab)  # RRUFF G1: 128 x 128 tiles (default) vs 64 x 64 (HPNN_TN_T64=1), 32 / 16 splits
      step t64_def 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_TN_T64=1 step t64_32 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_TN_T64=1 HPNN_SPLITS=16,16 step t64_16 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_TN_T64=1 HPNN_SPLITS=16,8 step t64_8 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      step t64_defb 200 python bench.py --model rruff --steps 100 --warmup 10 &&
      HPNN_TN_T64=1 step t64_32b 200 python bench.py --model rruff --steps 100 --warmup 10 ;;
    g0s)  # MNIST fused G0 split count in the step (tiles x splits <= 256 for co-residency)
      step g0s48 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_SPLITS=40,1,1 step g0s40 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_SPLITS=32,1,1 step g0s32 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_SPLITS=48,1,1 step g0s48x 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_SPLITS=40,1,1 step g0s40b 200 python bench.py --steps 200 --warmup 20 &&
      step g0s48b 200 python bench.py --steps 200 --warmup 20 ;;
    gsab)  # steps per HIP graph replay
      step gs20 200 python bench.py --steps 200 --warmup 20 --graph-steps 20 &&
      step gs50 200 python bench.py --steps 200 --warmup 20 --graph-steps 50 &&
      step gs100 200 python bench.py --steps 200 --warmup 20 --graph-steps 100 &&
      step gs20b 200 python bench.py --steps 200 --warmup 20 --graph-steps 20 &&
      step gs50b 200 python bench.py --steps 200 --warmup 20 --graph-steps 50 &&
      step gs100b 200 python bench.py --steps 200 --warmup 20 --graph-steps 100 ;;
    synthab)  # synthetic 8 x 4096 ANN: 64 x 64 underfill tiles on (default) / off
      step sy1 300 python bench.py --model synth --steps 20 --warmup 5 &&
      HPNN_TN_T64=0 step sy0 300 python bench.py --model synth --steps 20 --warmup 5 &&
      step sy1b 300 python bench.py --model synth --steps 20 --warmup 5 &&
      HPNN_TN_T64=0 step sy0b 300 python bench.py --model synth --steps 20 --warmup 5 ;;
    tradeab)  # tile front chain: lane-pair trade of 8-byte halves (HPNN_TILE_TRADE=1) vs plain stores (default)
      HPNN_TILE_TRADE=1 step tr1 200 python bench.py --steps 200 --warmup 20 &&
      step tr0 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_TILE_TRADE=1 step tr1b 200 python bench.py --steps 200 --warmup 20 &&
      step tr0b 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_TILE_TRADE=1 step tr1c 200 python bench.py --steps 200 --warmup 20 &&
      step tr0c 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_TILE_TRACE=1 step trace_tr0 200 python scripts/tile_trace.py ;;
    xordab)  # tile front X^T stage writes: per-lane-pair order (HPNN_TILE_XORD=1) vs row order (default)
      HPNN_TILE_XORD=1 step xo1 200 python bench.py --steps 200 --warmup 20 &&
      step xo0 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_TILE_XORD=1 step xo1b 200 python bench.py --steps 200 --warmup 20 &&
      step xo0b 200 python bench.py --steps 200 --warmup 20 &&
      HPNN_TILE_XORD=1 step xo1c 200 python bench.py --steps 200 --warmup 20 &&
      step xo0c 200 python bench.py --steps 200 --warmup 20 ;;
    tnr) step tn_rruff 200 python scripts/tn_rruff_bench.py --splits 4,8,16,32 ;;
    widetr) HPNN_WIDE_TRACE=1 step wide_trace 200 python scripts/wide_bench.py ;;
    rehearse) step rehearse 400 bash scripts/gpu_rehearse.sh ;;
    learn) step learn 900 python scripts/learnability.py --out $O/learnability.jsonl ;;
    synthrs) step bench_synth_rs 300 python bench.py --model synth --grad-comm bf16rs --steps 20 --warmup 5 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo DONE
