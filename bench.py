#!/usr/bin/env python3
"""Headline benchmark: training samples/sec (whole node), MNIST 784-128-64-10 SNN.

Config (BASELINE.json): MNIST-shaped 784-128-64-10 softmax SNN, BF16 MFMA compute with FP32
accumulation / FP32 master weights, BPM (momentum 0.2, lr 0.01), batched mode (one fwd +
bwd + update per sample), synthetic data, random-init weights (reference init rule).
Weak scaling: every GPU trains on its own `--batch` samples per step; gradients are
all-reduced over RCCL (bucketed, overlapped with the backward).

--model rruff / synth runs the other GPU configs of BASELINE.json through the same
contract (RRUFF-shaped 4096-230-230 SNN, batch 16384 per GPU; synthetic 8 x 4096 ANN,
global batch 8192 split over the GPUs = strong scaling).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--model mnist|rruff|synth]
  N>1 is launched by the driver as
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ...
Prints ONE JSON line (rank 0).
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from hpnn_amd._lib import native  # noqa: E402
from hpnn_amd.models import MLP  # noqa: E402
from hpnn_amd.parallel import DataParallel, init_from_env  # noqa: E402

METRIC = "training samples/sec (whole node), MNIST 784-128-64-10 SNN at 1/2/4/8 MI355X"

# the other GPU configs of BASELINE.json (--model): sizes, type, batch, whether the batch is
# per GPU (weak scaling) or for the whole node (strong scaling), metric name
MODELS = {
    "mnist": ([784, 128, 64, 10], "SNN", 65536, "weak", METRIC,
              "mnist_snn 784-128-64-10 (SNN, BPM momentum 0.2, lr 0.01, batched mode)"),
    "rruff": ([4096, 230, 230], "SNN", 16384, "weak",
              "training samples/sec (whole node), RRUFF-XRD-shaped 4096-230-230 SNN",
              "rruff_snn 4096-230-230 (SNN, BPM momentum 0.2, lr 0.01, batched mode)"),
    "synth": ([4096] * 9, "ANN", 8192, "strong",
              "training samples/sec (whole node), synthetic 8-layer x 4096-wide ANN, global batch 8192",
              "synth_ann 4096^9 (ANN, BPM momentum 0.2, lr 0.01, batched mode)"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", choices=sorted(MODELS), default="mnist",
                    help="mnist: the headline config; rruff / synth: the other BASELINE.json GPU configs")
    ap.add_argument("--batch", type=int, default=0,
                    help="per-GPU minibatch (default: the config's; synth splits its global 8192 over the GPUs)")
    ap.add_argument("--datasets", type=int, default=4, help="distinct synthetic minibatches cycled per GPU")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--alpha", type=float, default=0.2)
    ap.add_argument("--graph", type=int, default=1,
                    help="capture the steps in HIP graphs (0: eager, 2: also with torch.distributed collectives)")
    ap.add_argument("--graph-steps", type=int, default=20, help="training steps per graph replay")
    ap.add_argument("--input", choices=["u8", "float"], default="u8",
                    help="synthetic images as 8-bit pixels (MNIST's format; the net sees pixel/255 in BF16) "
                         "or as uniform floats in [0, 1)")
    ap.add_argument("--grad-comm", choices=["auto", "fp32", "bf16rs"], default="auto",
                    help="data-parallel gradient exchange: FP32 all-reduce, or BF16 reduce-scatter + sharded "
                         "optimizer step + BF16 weight all-gather (half the bytes; per-layer models only)")
    ap.add_argument("--settle-ms", type=float, default=50.0,
                    help="untimed steps for about this long before the warmup, so the timed steps see the GPU at "
                         "its steady clock (the first ~20 ms of steps after idle run 10-20%% slower; "
                         "profiles/r5/SUMMARY.md); 0: off")
    ap.add_argument("--eager-warmup", type=int, default=1,
                    help="1 (default): the W warmup steps as eager launches, so the run captures ONE graph -- a "
                         "second captured graph (W %% graph-steps steps) made the timed replay 4-5 us per step "
                         "slower on the GPU (profiles/r6/SUMMARY.md); 0: a graph of W %% graph-steps steps")
    ap.add_argument("--warmup-first", action="store_true",
                    help="the W warmup steps before the settle phase instead of after it (A/B: no measurable "
                         "difference, profiles/r6/SUMMARY.md)")
    ap.add_argument("--replay-trace", default="",
                    help="diagnostics: write the GPU time of every timed graph replay (ms) to this JSON file")
    args = ap.parse_args()

    # HPNN_BENCH_REHEARSE=1: rehearse the N > 1 path with several ranks on ONE GPU -- gloo
    # process group, gradients through the xGMI all-reduce kernel only (RCCL refuses two
    # ranks on one device); the timing is then meaningless, the code path is the driver's
    rehearse = os.environ.get("HPNN_BENCH_REHEARSE", "0") == "1"
    rank, world, local = init_from_env("gloo" if rehearse else None)
    if rehearse:
        local = 0
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    sizes, net, batch, scaling, metric, model_name = MODELS[args.model]
    if not args.batch:
        args.batch = batch // world if scaling == "strong" else batch
    # HPNN_SPLITS="s0,s1,..." (tuning only): per-layer split-K override of the plan
    sp = os.environ.get("HPNN_SPLITS")
    m = MLP(sizes, net, batch=args.batch, device=dev, momentum=True, seed=10958,
            init="reference" if args.model == "mnist" else "fast",
            splits=[int(v) for v in sp.split(",")] if sp else None)
    if rehearse and world > 1 and hasattr(m, "plan") and os.environ.get("HPNN_REHEARSE_FUSED", "0") != "1":
        # ranks sharing one GPU: the fused first-layer gradient needs all its workgroups
        # co-resident (in-kernel split-K reduction), which another rank's kernels on the same
        # CUs can prevent -- the rehearsal takes the slab form (one GPU per rank in real runs).
        # HPNN_REHEARSE_FUSED=1 keeps it, for per-rank batches whose grids fit together.
        m.plan.g0_fused = False
    dp = DataParallel(m, comm="xar" if rehearse and world > 1 else "auto",
                      grad_comm=args.grad_comm if m.fused_mode is None else "fp32")
    dp.broadcast_parameters()

    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    Xs, Ls = [], []
    for _ in range(args.datasets):
        if args.input == "u8" and args.model == "mnist":
            X = torch.randint(0, 256, (m.Bp, sizes[0]), device=dev, generator=g, dtype=torch.uint8)
        else:
            X = torch.rand(m.Bp, sizes[0], device=dev, generator=g)
        Xs.append(m.prepare_input(X))
        if net == "SNN":
            Ls.append(torch.randint(0, sizes[-1], (m.Bp,), device=dev, generator=g, dtype=torch.int32))
        else:  # ANN: dense +-1 targets of a random class
            T = torch.full((m.Bp, sizes[-1]), -1.0, device=dev)
            T[torch.arange(m.Bp, device=dev), torch.randint(0, sizes[-1], (m.Bp,), device=dev, generator=g)] = 1.0
            Ls.append(T)
    torch.cuda.synchronize()

    def step(i):
        tgt = Ls[i % args.datasets]
        kw = dict(labels=tgt) if net == "SNN" else dict(T=tgt)
        dp.train_step(Xs[i % args.datasets], lr=args.lr, alpha=args.alpha, **kw)

    # HIP graphs: single GPU always; data parallel when the gradient all-reduce goes through
    # libhpnn's native RCCL communicator (capturable: event fork/join of its side stream),
    # --graph 2 forces capture with torch.distributed collectives too
    use_graph = bool(args.graph) and (not dp.active or dp.native is not None or args.graph == 2)
    gsteps = max(1, args.graph_steps)
    if args.steps % gsteps and args.steps <= 5 * gsteps:
        gsteps = args.steps  # one graph for the timed steps (and the settle phase), no remainder graph
    graphs = {}

    def capture(n):
        """one HIP graph holding n consecutive training steps (cycling over the synthetic
        batches, whose input pointers are baked in): a replay launches n full steps, so the
        host-side replay gap is paid once per n steps"""
        if n not in graphs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(n):
                    step(i)
            graphs[n] = g
        return graphs[n]

    def leave_xgmi(why):
        """every rank stops using the xGMI exchange (collective: all ranks call it): RCCL takes
        the gradients, or torch.distributed when there is no RCCL communicator (rehearsal);
        the replicas restart from rank 0's weights (reference: the P2P -> CMM -> EXP fallback
        of libhpnn.c:245-302, decided once and agreed by every rank)"""
        nonlocal use_graph
        if rank == 0:
            print(f"{why}; falling back to {'RCCL' if dp.native.h else 'torch.distributed'}", file=sys.stderr)
        dp.native.detach_xar()
        if not dp.native.h:  # xGMI-only (rehearsal): torch.distributed takes the gradients
            # keep the detached communicator (and its IPC-mapped buffers) alive until every rank
            # is past the final barrier: a peer may still be inside a timed-out all-reduce
            # reading them
            dp._detached_native = dp.native
            dp.native = None
            use_graph = bool(args.graph) and args.graph == 2
        dp.broadcast_parameters()

    # one eager step first: when the xGMI all-reduce is in use, every rank checks that its
    # barriers completed and all ranks agree, else all fall back to RCCL before anything
    # is captured or timed
    step(0)
    torch.cuda.synchronize()
    if dp.native is not None and dp.native.xar:
        if not dp.all_ok(dp.native.xar_healthy()):
            leave_xgmi("xGMI all-reduce barrier timed out on some rank")

    # the replicas must hold bitwise-identical weights after the first exchange (a sum that
    # arrived in time but is wrong shows here, before anything is timed).  Over xGMI: degrade
    # to the next exchange, re-broadcast, one more step, check again; no result only if the
    # fallback disagrees too
    if dp.active and not dp.weights_consistent():
        if dp.native is not None and dp.native.xar:
            leave_xgmi("replica weights differ after the first step over xGMI")
            step(1)
            torch.cuda.synchronize()
        if not dp.weights_consistent():
            if rank == 0:
                print("replica weights differ after the first step; no result reported", file=sys.stderr)
            sys.exit(3)

    if use_graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for i in range(3):
                step(i)
        torch.cuda.current_stream().wait_stream(s)
        # capture every graph the run will replay before anything is timed; a capture
        # failure on any rank sends every rank back to eager steps (captured collectives
        # never ran, so the ranks stay in step)
        ok = True
        try:
            wn = 0 if args.eager_warmup else args.warmup % gsteps
            for n in {gsteps, args.steps % gsteps, wn} - {0}:
                capture(n)
        except Exception as e:  # noqa: BLE001
            ok = False
            print(f"rank {rank}: HIP graph capture failed ({e}); running eager steps", file=sys.stderr)
        torch.cuda.synchronize()
        if dp.active and not dp.all_ok(ok):
            ok = False
        if not ok:
            graphs.clear()
            use_graph = False

    marks = []  # --replay-trace: one event after each timed replay

    def run_steps(first, n, trace=False, eager=False):
        if use_graph and not eager:
            for _ in range(n // gsteps):
                graphs[gsteps].replay()
                if trace:
                    marks.append(torch.cuda.Event(enable_timing=True))
                    marks[-1].record()
            if n % gsteps:
                graphs[n % gsteps].replay()
        else:
            for i in range(first, first + n):
                step(i)

    # settle: whole steps for ~settle_ms (the same count on every rank: the steps hold
    # collectives), then the W warmup steps, then the K timed steps
    settle = 0
    if args.warmup_first:
        run_steps(0, args.warmup, eager=bool(args.eager_warmup))
    if args.settle_ms > 0:
        t_a = time.perf_counter()
        run_steps(0, gsteps)
        torch.cuda.synchronize()
        est = torch.tensor([(time.perf_counter() - t_a) / gsteps], dtype=torch.float64,
                           device="cpu" if rehearse else dev)
        if world > 1:
            dist.all_reduce(est, op=dist.ReduceOp.MAX)
        settle = gsteps * max(0, math.ceil(args.settle_ms * 1e-3 / max(float(est.item()), 1e-6) / gsteps) - 1)
        run_steps(gsteps, settle)
        settle += gsteps
    if not args.warmup_first:
        run_steps(0, args.warmup, eager=bool(args.eager_warmup))
    torch.cuda.synchronize()
    if world > 1 and rank == world - 1 and native().fault_hit("weights"):
        # test hook (HPNN_FAULT=weights:1): one replica's weights drift from the others'
        m.W32[0].view(-1)[0] += 1.0
        m.refresh_bf16()
    m.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.replay_trace:
        marks.append(torch.cuda.Event(enable_timing=True))
        marks[-1].record()
    run_steps(args.warmup, args.steps, bool(args.replay_trace))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    if args.replay_trace and rank == 0:
        with open(args.replay_trace, "w") as f:
            json.dump({"steps_per_replay": gsteps,
                       "replay_ms": [a.elapsed_time(b) for a, b in zip(marks, marks[1:])]}, f)
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device="cpu" if rehearse else dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    # timed-region integrity: a barrier timeout inside a replayed xGMI all-reduce, or an
    # asynchronous RCCL error, leaves wrong sums behind without stopping the ranks -- every
    # rank re-checks its communicator and all must agree, else no number is reported
    # in-kernel hand-offs (split-K tickets, tile pairs) must not have timed out: such a step
    # used partial sums -- checked at N = 1 too
    healthy = m.healthy()
    if not healthy:
        print(f"rank {rank}: an in-kernel hand-off timed out during the timed steps", file=sys.stderr)
    if dp.active:
        try:
            dp.check()
        except RuntimeError as e:
            print(f"rank {rank}: {e}", file=sys.stderr)
            healthy = False
        if dp.native is not None and not dp.native.xar_healthy():
            healthy = False
        healthy = dp.all_ok(healthy)
        if healthy and not dp.weights_consistent():
            print(f"rank {rank}: replica weights differ after the timed steps", file=sys.stderr)
            healthy = False
    if not healthy:
        if rank == 0:
            print("communication failed during the timed steps; no result reported", file=sys.stderr)
        if dp.active:
            dist.barrier()
        sys.exit(3)
    loss_sum, correct = m.read_stats()
    samples = args.steps * m.Bp * world
    value = samples / elapsed
    if rank == 0:
        u8 = args.input == "u8" and args.model == "mnist"
        out = {
            "metric": metric,
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_steps": settle,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "bf16",
            "data": ("synthetic (uniform 8-bit pixels 0..255 -> pixel/255 in BF16 as MNIST images, uniform labels; "
                     "random-init weights, reference init rule)" if u8 else
                     ("synthetic (uniform [0,1) pixels, uniform labels; random-init weights, reference init rule)"
                      if args.model == "mnist" else
                      "synthetic (uniform [0,1) inputs, uniform labels (SNN) / +-1 one-hot targets (ANN); "
                      "random-init weights)")),
            "config": {
                "model": model_name,
                "global_batch": m.Bp * world,
                "per_gpu_batch": m.Bp,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "hip_graph": bool(use_graph),
                "grad_allreduce": ("none" if not dp.active else
                                   (("xgmi+rccl" if dp.native.h else "xgmi") if dp.native is not None and dp.native.xar else
                                    ("rccl-native" if dp.native is not None else "torch.distributed"))),
                "grad_exchange": ("bf16 reduce-scatter + sharded update + bf16 all-gather" if dp.sharded else
                                  "fp32, inside the first-layer gradient launch"
                                  if getattr(dp, "xar_inplace", False) == "kernel" else "fp32"),
                "steps_per_graph": min(gsteps, args.steps) if use_graph else 0,
            },
            "train_loss_mean": loss_sum / max(1, samples // world),
        }
        emu = os.environ.get("HPNN_DPX_EMULATE_WORLD")
        if emu and dp.sharded:
            # one rank ran the sharded step at that world's per-rank sizes (timing only)
            out["config"]["dpx_emulated_world"] = int(emu)
        print(json.dumps(out))
    if dp.active:
        dist.barrier()
        if dp.native is not None:
            dp.native.close()
        if getattr(dp, "_detached_native", None) is not None:
            dp._detached_native.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
