#!/usr/bin/env python3
"""Throughput of the other BASELINE.json configs on ONE GPU (the headline MNIST config
is bench.py).  Prints one JSON line per config:
  rruff_snn   : RRUFF-XRD-shaped 4096 -> 230 -> 230 SNN, BPM, batch 16384
  synth_ann   : synthetic 8-layer x 4096-wide ANN (4096^9 sizes), BPM, batch 8192 (the
                8-GPU config's global batch on one GPU; per-GPU work at 8 GPUs is 1/8)
  ann484_cpu  : 4-8-4 ANN regression through the C API on the FP64 CPU engine
Synthetic data, random-init weights; steps captured in HIP graphs like bench.py.
usage: python scripts/bench_configs.py [--steps K] [--only NAME]"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hpnn_amd.models import MLP  # noqa: E402


def gpu_config(name, sizes, net, batch, steps, warmup=3):
    dev = torch.device("cuda")
    m = MLP(sizes, net, batch=batch, device=dev, momentum=True, seed=7, init="fast")
    g = torch.Generator(device=dev).manual_seed(5)
    X = m.prepare_input(torch.rand(m.Bp, sizes[0], device=dev, generator=g))
    if net == "SNN":
        L = torch.randint(0, sizes[-1], (m.Bp,), device=dev, generator=g, dtype=torch.int32)
        kw = dict(labels=L)
    else:
        T = torch.rand(m.Bp, sizes[-1], device=dev, generator=g) * 2 - 1
        kw = dict(T=T)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warmup):
            m.train_step(X, lr=0.001, alpha=0.2, **kw)
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        m.train_step(X, lr=0.001, alpha=0.2, **kw)
    for _ in range(warmup):
        gr.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        gr.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    P = sum(sizes[i] * sizes[i + 1] for i in range(len(sizes) - 1))
    flop = 6 * P - 2 * sizes[0] * sizes[1]  # fwd 2P + dW 2P + dX 2(P - first layer)
    return {"config": name, "sizes": sizes, "type": net, "batch": m.Bp, "ms_per_step": dt * 1e3,
            "samples_per_s": m.Bp / dt, "tflops": flop * m.Bp / dt / 1e12, "dtype": "bf16", "n_gpus": 1,
            "data": "synthetic", "fused_path": m.fused_mode}


def cpu_ann484(steps):
    from hpnn_amd import capi
    lib = capi.lib()
    d = tempfile.mkdtemp()
    sd = os.path.join(d, "samples")
    os.mkdir(sd)
    g = torch.Generator().manual_seed(3)
    n = 32
    for i in range(n):
        x = torch.rand(4, generator=g, dtype=torch.float64) * 2 - 1
        t = torch.tanh(x.flip(0))
        with open(os.path.join(sd, f"s{i:05d}.txt"), "w") as f:
            f.write("[input] 4\n" + " ".join(f"{v:.6f}" for v in x) + "\n[output] 4\n" +
                    " ".join(f"{v:.6f}" for v in t) + "\n")
    conf = os.path.join(d, "nn.conf")
    with open(conf, "w") as f:
        f.write(f"[name] ann484\n[type] ANN\n[init] generate\n[seed] 10958\n[input] 4\n[hidden] 8\n[output] 4\n"
                f"[train] BP\n[sample_dir] {sd}\n[test_dir] {sd}\n")
    capi.init(0)
    net = capi.Network(conf)
    net.set(device="cpu")  # FP64 CPU engine
    t0 = time.perf_counter()
    for _ in range(steps):
        net.train()
    dt = time.perf_counter() - t0
    capi.deinit()
    return {"config": "ann484_cpu", "sizes": [4, 8, 4], "type": "ANN", "mode": "online (reference loop)",
            "samples_per_s": steps * n / dt, "engine": "FP64 CPU", "data": "synthetic"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    todo = [("rruff_snn", lambda: gpu_config("rruff_snn", [4096, 230, 230], "SNN", 16384, a.steps)),
            ("synth_ann", lambda: gpu_config("synth_ann", [4096] * 9, "ANN", 8192, max(3, a.steps // 4))),
            ("ann484_cpu", lambda: cpu_ann484(1))]
    for name, fn in todo:
        if a.only and name != a.only:
            continue
        try:
            print(json.dumps(fn()), flush=True)
        except Exception as e:  # report and continue with the other configs
            print(json.dumps({"config": name, "error": repr(e)}), flush=True)


if __name__ == "__main__":
    main()
