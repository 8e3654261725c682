"""Per-step time of the library's batched engine (train_nn -m batched, the reference's entry
point: tests/train_nn.c:232 -> nn_train_kernel) against bench.py for the same configs.

Both drive the same plan (csrc/gpu/bplan.h).  train_nn trains `--batches` minibatches per
epoch for `--epochs` epochs from a generated pack file (8-bit pixel values for the MNIST
shape, uniform floats for RRUFF) and prints its training wall time; per step = seconds /
(epochs x batches).  bench.py runs its usual timed loop.  Writes one JSON line per config.

    python scripts/lib_vs_bench.py --out gpurun_out/lib_vs_bench.jsonl
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hpnn_amd import capi  # noqa: E402
from hpnn_amd.utils import formats  # noqa: E402

CONFIGS = {"mnist": ((784, [128, 64], 10), 65536, True), "rruff": ((4096, [230], 230), 16384, False),
           # FP64 / FP32 only (no bench.py counterpart): 4096-wide hidden layers
           "wide": ((4096, [4096, 4096], 10), 4096, False)}


def run_train_nn(name, batches, epochs, work, dtype="bf16", dpforce=False):
    (n_in, hid, n_out), B, pixels = CONFIGS[name]
    n = B * batches
    rng = np.random.default_rng(3)
    X = rng.integers(0, 256, (n, n_in), dtype=np.uint8).astype(np.float64) if pixels else \
        rng.uniform(0, 1, (n, n_in)).astype(np.float64)
    T = np.zeros((n, n_out))
    T[np.arange(n), rng.integers(0, n_out, n)] = 1.0
    d = os.path.join(work, name)
    os.makedirs(d, exist_ok=True)
    capi.pack_arrays(os.path.join(d, "train.hpnb"), X, T)
    del X, T
    formats.write_conf(os.path.join(d, "nn.conf"), name=name, type="SNN", seed=10958, inputs=n_in, hiddens=hid,
                       outputs=n_out, train="BPM", sample_dir="./train.hpnb", test_dir="./train.hpnb",
                       mode="batched", batch=B, epochs=epochs, dtype=dtype, lr=0.01)
    env = dict(os.environ)
    env.pop("HPNN_FORCE_CPU", None)
    if dpforce:  # the N > 1 path (train_dp_mp) with one rank, as under `torchrun --no-python`
        env.update(HPNN_DP_FORCE="1", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
                   HPNN_BOOT_DIR=os.path.join(work, "boot"))
    r = subprocess.run([os.path.join(ROOT, "bin", "train_nn"), "-vvv", "nn.conf"], cwd=d, env=env,
                       capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise SystemExit(r.stdout[-3000:] + r.stderr[-3000:])
    m = re.search(r"BATCHED TRAINING: (\d+) samples in ([0-9.]+) s", r.stdout)
    mode = re.search(r"batched plan: mode (\S)", r.stdout)
    if dpforce and "data-parallel epochs: HIP graph replays" not in r.stdout:
        raise SystemExit("train_nn did not replay HIP graphs on the data-parallel path:\n" + r.stdout[-3000:])
    samples, secs = int(m.group(1)), float(m.group(2))
    steps = epochs * batches
    rec = {"us_per_step": secs / steps * 1e6, "steps": steps, "samples": samples, "seconds": secs,
           "plan_mode": mode.group(1) if mode else None}
    e1 = re.search(r"epoch 1 \(eager, with the weight digest\) ([0-9.]+) ms", r.stdout)
    if e1:
        rec["first_epoch_ms"] = float(e1.group(1))
    return rec


def run_bench(name, steps, dpforce=False):
    # no settle phase: train_nn's timed epochs start from an idle GPU too (the same clock ramp)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--model", name, "--steps", str(steps), "--warmup", "10",
           "--settle-ms", "0"]
    env = dict(os.environ)
    if dpforce:
        env["HPNN_DP_FORCE"] = "1"
        cmd[1:1] = ["-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1", "--master-addr",
                    "127.0.0.1", "--master-port", "29677"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    if r.returncode != 0:
        raise SystemExit(r.stdout[-3000:] + r.stderr[-3000:])
    j = json.loads(r.stdout.strip().splitlines()[-1])
    return {"us_per_step": j["ms_per_step"] * 1e3, "steps": steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="mnist,rruff")
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--dtype", default="bf16", help="bf16 (compared with bench.py) | f32 | f64 (train_nn only)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--dpforce", action="store_true",
                    help="both on the N > 1 path with one rank (HPNN_DP_FORCE=1 under a launcher)")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as work:
        for name in a.configs.split(","):
            lib = run_train_nn(name, a.batches, a.epochs, work, a.dtype, a.dpforce)
            rec = {"config": name, "dtype": a.dtype, "batch": CONFIGS[name][1], "train_nn": lib,
                   "path": "dp (one rank)" if a.dpforce else "single"}
            if a.dtype == "bf16":
                b = run_bench(name, 200, a.dpforce)
                rec.update(bench=b, ratio=round(lib["us_per_step"] / b["us_per_step"], 4))
            else:
                (n_in, hid, n_out), B, _ = CONFIGS[name]
                dims = [n_in] + hid + [n_out]
                flops = 6.0 * B * sum(dims[i] * dims[i + 1] for i in range(len(dims) - 1))
                rec["step_tflops"] = round(flops / (lib["us_per_step"] * 1e-6) / 1e12, 2)
            print(json.dumps(rec), flush=True)
            if a.out:
                with open(a.out, "a") as f:
                    f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
