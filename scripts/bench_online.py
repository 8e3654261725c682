#!/usr/bin/env python3
"""Online (reference-semantics) training throughput: train_nn in online mode on the GPU
engine (one persistent FP64 kernel per sample) vs the FP64 CPU engine, MNIST-tutorial
shapes (784-300-10 ANN BP, 784-128-64-10 SNN BPM).  Synthetic samples (uniform pixels in
[0,1), random one-hot).  usage: python scripts/bench_online.py [--n 200] [--cpu-n 20]"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hpnn_amd.utils import formats  # noqa: E402


def run(d, n, net, hid, train, cpu):
    s = os.path.join(d, "s")
    os.makedirs(s, exist_ok=True)
    rng = np.random.default_rng(0)
    for i in range(n):
        t = np.full(10, 0.0 if net == "SNN" else -1.0)
        t[int(rng.integers(10))] = 1.0
        formats.write_sample(os.path.join(s, f"s{i:05d}.txt"), rng.random(784), t)
    formats.write_conf(os.path.join(d, "nn.conf"), name="o", type=net, seed=10958, inputs=784, hiddens=hid,
                       outputs=10, train=train, sample_dir="./s", test_dir="./s")
    env = dict(os.environ)
    if cpu:
        env["HPNN_FORCE_CPU"] = "1"
    t0 = time.perf_counter()
    r = subprocess.run([os.path.join(ROOT, "bin", "train_nn"), "-vv", "-x", "nn.conf"], cwd=d, env=env,
                       capture_output=True, text=True, timeout=1800)
    dt = time.perf_counter() - t0
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    its = [int(m) for m in re.findall(r"N_ITER=\s*(\d+)", r.stdout)]
    return {"net": f"{net} 784-{'-'.join(map(str, hid))}-10 {train}", "engine": "FP64 CPU" if cpu else "GPU online",
            "samples": len(its), "seconds": dt, "samples_per_s": len(its) / dt,
            "mean_iterations": sum(its) / max(1, len(its)), "iterations_per_s": sum(its) / dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--cpu-n", type=int, default=20)
    a = ap.parse_args()
    for net, hid, train in (("ANN", [300], "BP"), ("SNN", [128, 64], "BPM")):
        for cpu in (False, True):
            with tempfile.TemporaryDirectory() as d:
                print(json.dumps(run(d, a.cpu_n if cpu else a.n, net, hid, train, cpu)), flush=True)


if __name__ == "__main__":
    main()
