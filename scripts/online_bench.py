"""Iterations/s of the FP64 online engine (reference semantics: one sample at a time, the
convergence loop of fwd + bwd + update until the error stops improving) on a wide net.

Writes N random samples, runs bin/train_nn with HPNN_METRICS, and takes the per-sample
timestamps and N_ITER values from the metrics JSONL: it/s = sum(n_iter) / elapsed over
samples 2..N (sample 1 pays the device setup).  Each configuration in --env runs in its own
train_nn process; its comma-separated items are VAR=value pairs or train_nn flags ("-S2").

    python scripts/online_bench.py --dims 4096,4096,230 --n 6 --env '' --env HPNN_ONLINE_SLOTS=2 --env=-S2
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hpnn_amd.utils import formats  # noqa: E402


def run(dims, n, train, net, env_s, work):
    n_in, hid, n_out = dims[0], dims[1:-1], dims[-1]
    d = os.path.join(work, (env_s or "default").replace("=", "_"))
    os.makedirs(os.path.join(d, "samples"), exist_ok=True)
    rng = np.random.default_rng(1)
    for i in range(n):
        x = rng.uniform(0, 1, n_in)
        t = np.full(n_out, 0.0 if net == "SNN" else -1.0)
        t[int(rng.integers(n_out))] = 1.0
        formats.write_sample(os.path.join(d, "samples", f"s{i:05d}.txt"), x, t)
    formats.write_conf(os.path.join(d, "nn.conf"), name="wide", type=net, seed=3, inputs=n_in, hiddens=hid,
                       outputs=n_out, train=train, sample_dir="./samples", test_dir="./samples", lr=0.001)
    env = dict(os.environ, HPNN_METRICS="m.jsonl")
    env.pop("HPNN_FORCE_CPU", None)
    flags = []
    for kv in filter(None, env_s.split(",")):
        if kv.startswith("-"):
            flags.append(kv)
            continue
        k, v = kv.split("=", 1)
        env[k] = v
    r = subprocess.run([os.path.join(ROOT, "bin", "train_nn"), "-v"] + flags + ["nn.conf"], cwd=d, env=env,
                       capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise SystemExit(r.stdout[-2000:] + r.stderr[-2000:])
    ev = [json.loads(l) for l in open(os.path.join(d, "m.jsonl"))]
    smp = [e for e in ev if e["event"] == "train_sample"]
    its = sum(e["n_iter"] for e in smp[1:])
    dt = smp[-1]["time"] - smp[0]["time"]
    return {"env": env_s or "(one device)", "dims": dims, "train": train, "samples_timed": len(smp) - 1,
            "iterations": its, "seconds": round(dt, 6), "it_per_s": round(its / dt, 2) if dt > 0 else None,
            "ms_per_iter": round(1e3 * dt / its, 4) if its else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dims", default="4096,4096,230")
    ap.add_argument("--n", type=int, default=6)
    ap.add_argument("--train", default="BPM")
    ap.add_argument("--net", default="SNN")
    ap.add_argument("--env", action="append", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dims = [int(v) for v in a.dims.split(",")]
    res = []
    with tempfile.TemporaryDirectory() as work:
        for env_s in a.env or [""]:
            r = run(dims, a.n, a.train, a.net, env_s, work)
            print(json.dumps(r), flush=True)
            res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
