#!/usr/bin/env python3
"""Learnability record: the batched engines trained end to end (train_nn -m batched, then
run_nn on held-out samples) on synthetic labelled data a correct engine learns to a high
test accuracy and a broken one cannot (no dataset can be downloaded here).

    data      10 fixed random prototypes p_c in [0, 1]^784; a sample of class c is
              clip(p_c + N(0, sigma^2), 0, 1), sigma = 2 (pixel-like images, noise larger than
              the signal in every pixel)
    student   SNN 784-128-64-10 (the BASELINE net), BPM, minibatch 256

Engines: "gpu" = the BF16 batched engine on the GPU (the fused MNIST plan), "cpu" = the FP64
batched CPU engine (HPNN_FORCE_CPU=1, [dtype] f64: the reference's precision).  One JSON
record per engine (test accuracy, per-epoch training loss / accuracy from HPNN_METRICS).

    python scripts/learnability.py --engines gpu,cpu --out profiles/r4/learnability.jsonl
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hpnn_amd import capi  # noqa: E402
from hpnn_amd.utils import formats  # noqa: E402

BIN = os.path.join(ROOT, "bin")


def prototype_data(n, seed, n_in=784, n_out=10, noise=1.0):
    """class c has a fixed random prototype p_c in [0, 1]^784; a sample of class c is
    clip(p_c + N(0, noise^2), 0, 1) (pixel-like, heavily corrupted: most single pixels say
    little about the class, the whole image does)"""
    rng = np.random.default_rng(1234)  # the prototypes are fixed
    protos = rng.uniform(0.0, 1.0, (n_out, n_in))
    r = np.random.default_rng(seed)
    lab = r.integers(0, n_out, n)
    X = np.clip(protos[lab] + r.normal(0.0, noise, (n, n_in)), 0.0, 1.0)
    T = np.zeros((n, n_out))
    T[np.arange(n), lab] = 1.0
    return X, T, lab


def run(engine, d, epochs, lr, batch, timeout):
    env = dict(os.environ)
    env.pop("HPNN_FORCE_CPU", None)
    if engine == "cpu":
        env["HPNN_FORCE_CPU"] = "1"
    env["HPNN_METRICS"] = os.path.join(d, f"metrics_{engine}.jsonl")
    conf = os.path.join(d, f"nn_{engine}.conf")
    formats.write_conf(conf, name=f"learn_{engine}", type="SNN", seed=7, inputs=784, hiddens=[128, 64], outputs=10,
                       train="BPM", sample_dir="./train.hpnb", test_dir="./test.hpnb", mode="batched", batch=batch,
                       epochs=epochs, lr=lr, dtype="bf16" if engine == "gpu" else "f64")
    t0 = time.time()
    r = subprocess.run([os.path.join(BIN, "train_nn"), "-v", conf], cwd=d, env=env, capture_output=True, text=True,
                       timeout=timeout)
    t_train = time.time() - t0
    if r.returncode:
        raise RuntimeError(r.stdout[-2000:] + r.stderr[-2000:])
    os.replace(os.path.join(d, "kernel.opt"), os.path.join(d, f"kernel_{engine}.opt"))
    formats.write_conf(conf, name=f"learn_{engine}", type="SNN", init=f"kernel_{engine}.opt", seed=7, inputs=784,
                       hiddens=[128, 64], outputs=10, train="BPM", sample_dir="./train.hpnb", test_dir="./test.hpnb",
                       mode="batched", batch=batch, dtype="bf16" if engine == "gpu" else "f64")
    r = subprocess.run([os.path.join(BIN, "run_nn"), "-v", conf], cwd=d, env=env, capture_output=True, text=True,
                       timeout=timeout)
    if r.returncode:
        raise RuntimeError(r.stdout[-2000:] + r.stderr[-2000:])
    traj, test = [], None
    with open(env["HPNN_METRICS"]) as f:
        for line in f:
            e = json.loads(line)
            if e.get("event") == "epoch":
                traj.append({k: e[k] for k in ("epoch", "loss", "accuracy") if k in e})
            elif e.get("event") == "run":
                test = e
    if test is None:
        raise RuntimeError("run_nn wrote no result: " + r.stdout[-2000:] + r.stderr[-2000:])
    return {"engine": engine, "dtype": "bf16" if engine == "gpu" else "f64", "test_accuracy": test["accuracy"],
            "n_test": test["total"], "train_seconds": round(t_train, 2), "epochs": traj}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engines", default="gpu,cpu")
    ap.add_argument("--n-train", type=int, default=60000)
    ap.add_argument("--n-test", type=int, default=10000)
    ap.add_argument("--epochs", type=int, default=8)
    ap.add_argument("--lr", type=float, default=0.2)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--timeout", type=int, default=1800)
    ap.add_argument("--noise", type=float, default=2.0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        X, T, lab = prototype_data(a.n_train, 1, noise=a.noise)
        capi.pack_arrays(os.path.join(d, "train.hpnb"), X, T)
        Xt, Tt, labt = prototype_data(a.n_test, 2, noise=a.noise)
        capi.pack_arrays(os.path.join(d, "test.hpnb"), Xt, Tt)
        prior = float(np.bincount(labt, minlength=10).max() / len(labt))
        for eng in a.engines.split(","):
            rec = run(eng, d, a.epochs, a.lr, a.batch, a.timeout)
            rec.update({"net": "SNN 784-128-64-10 BPM", "batch": a.batch, "lr": a.lr, "n_train": a.n_train,
                        "data": f"10 noisy random prototypes, sigma {a.noise}, clipped to [0,1]", "majority_class_rate": prior})
            print(json.dumps(rec), flush=True)
            if a.out:
                with open(a.out, "a") as f:
                    f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
