"""Auxiliary subsystems through the native CLIs (CPU engine, HPNN_FORCE_CPU=1):

- exact checkpoint / resume (csrc/core/state.cpp): 2 epochs in one run == 1 epoch, state
  dump, 1 more epoch resumed from the state -- byte-identical state files and kernels;
  a corrupted state is refused (checksum);
- sample packs (csrc/core/dataset.cpp, bin/pack_nn): training from a pack == training
  from the directory; a corrupted pack is refused;
- metrics (HPNN_METRICS / -M): JSON-lines records per epoch / sample / run;
- tracing (-T / HPNN_TRACE): the timing table lists the driver ranges.

The reference has none of these; there is nothing to pin parity to beyond the
training math, which test_capi_cpu.py covers."""
import json
import os
import subprocess

import numpy as np
import pytest

from hpnn_amd.utils import formats

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


def _env(**kw):
    e = dict(os.environ)
    e["HPNN_FORCE_CPU"] = "1"
    e.update(kw)
    return e


def _run(cmd, cwd, ok=True, **kw):
    r = subprocess.run(cmd, cwd=cwd, env=_env(**kw), capture_output=True, text=True, timeout=300)
    if ok:
        assert r.returncode == 0, r.stdout + r.stderr
    return r


def _dataset(d, n=24, n_in=6, n_out=3, seed=2):
    rng = np.random.default_rng(seed)
    os.makedirs(d, exist_ok=True)
    for i in range(n):
        x = rng.uniform(-1, 1, n_in)
        t = np.zeros(n_out)
        t[int(np.argmax(x[:n_out]))] = 1.0
        formats.write_sample(os.path.join(d, f"s{i:04d}.txt"), x, t)


def _conf(d, samples="./samples", **kw):
    formats.write_conf(os.path.join(d, "nn.conf"), name="aux", type="SNN", seed=77, inputs=6, hiddens=[8],
                       outputs=3, train="BPM", sample_dir=samples, test_dir=samples, **kw)


def _read(p):
    with open(p, "rb") as f:
        return f.read()


def test_state_resume_is_exact(tmp_path):
    a, b = tmp_path / "a", tmp_path / "b"
    for d in (a, b):
        _dataset(str(d / "samples"))
        _conf(str(d))
    _run([os.path.join(BIN, "train_nn"), "-b", "5", "-e", "2", "-r", "state.bin", "nn.conf"], str(a))
    _run([os.path.join(BIN, "train_nn"), "-b", "5", "-e", "1", "-r", "state.bin", "nn.conf"], str(b))
    assert _read(b / "state.bin") != _read(a / "state.bin")
    out = _run([os.path.join(BIN, "train_nn"), "-vv", "-b", "5", "-e", "1", "-r", "state.bin", "nn.conf"],
               str(b)).stdout
    assert "1 epochs done" in out and "momentum restored" in out
    # same weights, momentum and progress counters, bit for bit
    assert _read(b / "state.bin") == _read(a / "state.bin")
    assert _read(b / "kernel.opt") == _read(a / "kernel.opt")


def test_state_corruption_is_detected(tmp_path):
    d = str(tmp_path)
    _dataset(os.path.join(d, "samples"))
    _conf(d)
    _run([os.path.join(BIN, "train_nn"), "-b", "5", "-r", "state.bin", "nn.conf"], d)
    raw = bytearray(_read(os.path.join(d, "state.bin")))
    raw[len(raw) // 2] ^= 0x40
    with open(os.path.join(d, "state.bin"), "wb") as f:
        f.write(raw)
    r = _run([os.path.join(BIN, "train_nn"), "-b", "5", "-r", "state.bin", "nn.conf"], d, ok=False)
    assert r.returncode != 0
    assert "checksum" in r.stdout + r.stderr


@pytest.mark.parametrize("mode", ["batched", "online"])
def test_pack_matches_directory(tmp_path, mode):
    a, b = tmp_path / "a", tmp_path / "b"
    _dataset(str(a / "samples"))
    _dataset(str(b / "samples"))
    _run([os.path.join(BIN, "pack_nn"), "samples", "train.hpnb"], str(b))
    _conf(str(a))
    _conf(str(b), samples="./train.hpnb")
    flags = ["-b", "4", "-e", "2"] if mode == "batched" else []
    oa = _run([os.path.join(BIN, "train_nn"), "-vv"] + flags + ["nn.conf"], str(a)).stdout
    ob = _run([os.path.join(BIN, "train_nn"), "-vv"] + flags + ["nn.conf"], str(b)).stdout
    assert _read(a / "kernel.opt") == _read(b / "kernel.opt")
    if mode == "online":
        # same per-sample log lines, file names included
        la = [ln for ln in oa.splitlines() if "TRAINING FILE" in ln]
        lb = [ln for ln in ob.splitlines() if "TRAINING FILE" in ln]
        assert la == lb and len(la) == 24
    ra = _run([os.path.join(BIN, "run_nn"), "-vv", "nn.conf"], str(a)).stdout
    rb = _run([os.path.join(BIN, "run_nn"), "-vv", "nn.conf"], str(b)).stdout
    assert ra.count("[PASS]") == rb.count("[PASS]") and ra.count("TESTING FILE") == 24


def test_pack_corruption_is_detected(tmp_path):
    d = str(tmp_path)
    _dataset(os.path.join(d, "samples"))
    _run([os.path.join(BIN, "pack_nn"), "samples", "p.hpnb"], d)
    raw = bytearray(_read(os.path.join(d, "p.hpnb")))
    raw[-20] ^= 0x01
    with open(os.path.join(d, "p.hpnb"), "wb") as f:
        f.write(raw)
    _conf(d, samples="./p.hpnb")
    r = _run([os.path.join(BIN, "train_nn"), "-b", "4", "nn.conf"], d, ok=False)
    assert r.returncode != 0 and "checksum" in r.stdout + r.stderr


def test_metrics_and_trace(tmp_path):
    d = str(tmp_path)
    _dataset(os.path.join(d, "samples"))
    _conf(d)
    out = _run([os.path.join(BIN, "train_nn"), "-T", "-b", "5", "-e", "3", "-M", "m.jsonl", "nn.conf"], d).stdout
    assert "NN(TRACE)" in out and "nn_train_kernel" in out and "load_samples" in out
    _run([os.path.join(BIN, "run_nn"), "nn.conf"], d, HPNN_METRICS="m.jsonl")
    _run([os.path.join(BIN, "train_nn"), "nn.conf"], d, HPNN_METRICS="m.jsonl")
    recs = [json.loads(ln) for ln in open(os.path.join(d, "m.jsonl"))]
    ev = [r["event"] for r in recs]
    assert ev[:4] == ["epoch", "epoch", "epoch", "train_batched"]
    assert [r["epoch"] for r in recs[:3]] == [1, 2, 3]
    assert all(r["loss"] > 0 and r["n"] == 24 for r in recs[:3])
    assert recs[3]["epochs_done"] == 3 and recs[3]["samples"] == 72
    assert "run" in ev and ev.count("train_sample") == 24 and ev[-1] == "train_online"
    run = recs[ev.index("run")]
    assert run["total"] == 24 and 0 <= run["pass"] <= 24


def test_python_state_pack_trace(tmp_path, monkeypatch):
    """the same subsystems through the ctypes binding (hpnn_amd.capi, hpnn_amd.utils.trace)"""
    from hpnn_amd import capi
    from hpnn_amd.utils import trace
    d = str(tmp_path)
    _dataset(os.path.join(d, "samples"))
    capi.pack_samples(os.path.join(d, "samples"), os.path.join(d, "p.hpnb"))
    _conf(d, samples=os.path.join(d, "p.hpnb"))
    monkeypatch.setenv("HPNN_FORCE_CPU", "1")
    capi.init(0)
    trace.enable(True)
    trace.reset()
    net = capi.Network(os.path.join(d, "nn.conf")).set(mode="batched", batch=6, epochs=2)
    with trace.phase("py.train"):
        assert net.train()
    assert net.epochs_done == 2
    net.dump_state(os.path.join(d, "s.bin"))
    w = _read(os.path.join(d, "s.bin"))
    net2 = capi.Network(os.path.join(d, "nn.conf"))
    net2.load_state(os.path.join(d, "s.bin"))
    assert net2.epochs_done == 2
    net2.dump_state(os.path.join(d, "s2.bin"))
    assert _read(os.path.join(d, "s2.bin")) == w
    rep = trace.report()
    assert rep["py.train"][0] == 1 and rep["nn_train_kernel"][0] == 1
    assert rep["py.train"][1] >= rep["nn_train_kernel"][1]
    trace.enable(False)
    net.close()
    net2.close()


def test_pack_arrays_matches_directory(tmp_path):
    """nn_pack_arrays (records from memory, e.g. a generated benchmark set) writes the same
    pack as the directory path: training from it gives the same kernel"""
    from hpnn_amd import capi
    a, b = tmp_path / "a", tmp_path / "b"
    _dataset(str(a / "samples"))
    files = sorted(os.listdir(a / "samples"))
    recs = [formats.read_sample(str(a / "samples" / f)) for f in files]
    os.makedirs(b, exist_ok=True)
    capi.pack_arrays(str(b / "gen.hpnb"), np.array([x for x, _ in recs]), np.array([t for _, t in recs]))
    _conf(str(a))
    _conf(str(b), samples="./gen.hpnb")
    for d in (a, b):
        _run([os.path.join(BIN, "train_nn"), "-vv", "-b", "4", "-e", "2", "nn.conf"], str(d))
    assert _read(a / "kernel.opt") == _read(b / "kernel.opt")
