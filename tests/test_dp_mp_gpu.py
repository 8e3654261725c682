"""Native multi-process data parallelism of train_nn (csrc/gpu/gpu_engine.cpp::train_dp_mp):
two train_nn processes launched like `torchrun --no-python` would (RANK / WORLD_SIZE /
LOCAL_RANK / LOCAL_WORLD_SIZE), both on the box's single MI355X, exchanging gradients
through the one-shot xGMI all-reduce and their bootstrap data through files -- the
reference's `mpirun -np 2 train_nn`.  The result equals one process training the same
global minibatches (FP32 summation order aside); rank 0 alone writes the files."""
import os
import socket
import subprocess

import numpy as np
import pytest

from hpnn_amd.utils import formats

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TN = os.path.join(ROOT, "bin", "train_nn")


def _data(d, n, n_in, n_out):
    rng = np.random.default_rng(1)
    os.makedirs(d, exist_ok=True)
    for i in range(n):
        t = np.zeros(n_out)
        t[int(rng.integers(n_out))] = 1.0
        formats.write_sample(os.path.join(d, f"s{i:05d}.txt"), rng.random(n_in), t)


def _env(**kw):
    e = dict(os.environ)
    for k in ("HPNN_FORCE_CPU", "HPNN_LOOPBACK_RANKS", "HPNN_FORCE_RCCL", "RANK", "WORLD_SIZE", "LOCAL_RANK",
              "LOCAL_WORLD_SIZE"):
        e.pop(k, None)
    e.update({k: str(v) for k, v in kw.items()})
    return e


@pytest.mark.gpu
@pytest.mark.parametrize("dims,dtype", [((784, [128, 64], 10), "bf16"), ((100, [48], 7), "bf16"),
                                        ((100, [48], 7), "f32")])
def test_train_nn_two_processes_equals_one(gpu, tmp_path, dims, dtype):
    n_in, hid, n_out = dims
    for sub in ("one", "two"):
        d = tmp_path / sub
        _data(str(d / "s"), 700, n_in, n_out)
        formats.write_conf(str(d / "nn.conf"), name="mp", type="SNN", seed=4, inputs=n_in, hiddens=hid, outputs=n_out,
                           train="BPM", sample_dir="./s", test_dir="./s", dtype=dtype)
    # MNIST-shaped: 256 samples per rank, the tile path (fused G0 with the in-kernel exchange)
    flags = ["-vv", "-b", "512" if n_in == 784 else "256", "-e", "2", "nn.conf"]
    r = subprocess.run([TN] + flags, cwd=tmp_path / "one", env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([TN] + flags, cwd=tmp_path / "two", stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True,
                              env=_env(RANK=r, WORLD_SIZE=2, LOCAL_RANK=0, LOCAL_WORLD_SIZE=2, MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=port, HPNN_BOOT_DIR=str(tmp_path / "boot"),
                                       HPNN_BOOT_TIMEOUT_S=60, HPNN_XAR_TIMEOUT_MS=3000))
             for r in range(2)]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=200)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    for rc, o, e in outs:
        assert rc == 0, o[-2000:] + e[-2000:]
    assert f"2 processes (xGMI all-reduce, {dtype})" in outs[0][1]
    assert "data-parallel epochs: HIP graph replays" in outs[0][1], outs[0][1][-2000:]
    if dims[0] == 784 and dtype == "bf16":  # fused tile mode: the exchange runs in the G0 launch
        assert "exchange inside the first-layer gradient launch" in outs[0][1], outs[0][1][-2000:]
    assert outs[1][1].strip() == ""  # rank 1 prints nothing
    w1 = formats.read_kernel(str(tmp_path / "one" / "kernel.opt"))["weights"]
    w2 = formats.read_kernel(str(tmp_path / "two" / "kernel.opt"))["weights"]
    for a, b in zip(w1, w2):
        assert np.abs(a - b).max() < 2e-5, np.abs(a - b).max()
    assert not os.listdir(tmp_path / "boot") or all(f.split(".")[0].isdigit() for f in os.listdir(tmp_path / "boot"))
