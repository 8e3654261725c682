"""Native engines on the GPU (train_nn / run_nn through libhpnn) vs the FP64 CPU engine."""
import os
import subprocess

import numpy as np
import pytest

from hpnn_amd.utils import formats

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


def _run(cmd, cwd, cpu=False, extra_env=None):
    env = dict(os.environ)
    env.pop("HPNN_LOOPBACK_RANKS", None)
    env.pop("HPNN_FORCE_RCCL", None)
    env.update(extra_env or {})
    if cpu:
        env["HPNN_FORCE_CPU"] = "1"
    else:
        env.pop("HPNN_FORCE_CPU", None)
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def _data(d, n, n_in, n_out, snn, seed=0):
    rng = np.random.default_rng(seed)
    os.makedirs(d, exist_ok=True)
    for i in range(n):
        x = rng.uniform(0, 1, n_in)
        t = np.full(n_out, 0.0 if snn else -1.0)
        t[int(rng.integers(n_out))] = 1.0
        formats.write_sample(os.path.join(d, f"s{i:05d}.txt"), x, t)


@pytest.mark.parametrize("net,train,dims", [("SNN", "BP", (40, [24, 16], 5)), ("ANN", "BPM", (40, [24, 16], 5)),
                                            ("SNN", "BPM", (120, [64, 40], 10)), ("ANN", "BP", (90, [300], 10)),
                                            ("ANN", "BPM", (70, [48, 200, 33], 7))])
def test_online_gpu_matches_cpu(tmp_path, net, train, dims):
    """FP64 online engines == FP64 CPU engine (reference semantics).  The small net runs the
    single-workgroup kernel, the wider ones the cooperative multi-workgroup kernel (rows
    dealt to resident workgroups, delta partials summed in workgroup order)."""
    n_in, hid, n_out = dims
    for dev in ("cpu", "gpu"):
        d = str(tmp_path / dev)
        _data(os.path.join(d, "samples"), 3, n_in, n_out, net == "SNN")
        formats.write_conf(os.path.join(d, "nn.conf"), name="t", type=net, seed=5, inputs=n_in, hiddens=hid,
                           outputs=n_out, train=train, sample_dir="./samples", test_dir="./samples", lr=0.01)
        out = _run([os.path.join(BIN, "train_nn"), "-vv", "nn.conf"], d, cpu=(dev == "cpu"))
        assert out.count("TRAINING FILE") == 3
    kc = formats.read_kernel(str(tmp_path / "cpu" / "kernel.opt"))["weights"]
    kg = formats.read_kernel(str(tmp_path / "gpu" / "kernel.opt"))["weights"]
    for a, b in zip(kc, kg):
        assert np.abs(a - b).max() < 1e-9, np.abs(a - b).max()


def test_batched_gpu_fused_close_to_cpu(tmp_path):
    """native batched engine on the GPU (fused MNIST-shaped path, BF16 MFMA) vs FP64 CPU."""
    res = {}
    for dev in ("cpu", "gpu"):
        d = str(tmp_path / dev)
        _data(os.path.join(d, "samples"), 300, 784, 10, True)
        formats.write_conf(os.path.join(d, "nn.conf"), name="m", type="SNN", seed=9, inputs=784, hiddens=[128, 64],
                           outputs=10, train="BPM", sample_dir="./samples", test_dir="./samples", mode="batched",
                           batch=128, epochs=2, lr=0.05, dtype="bf16")
        _run([os.path.join(BIN, "train_nn"), "-vv", "nn.conf"], d, cpu=(dev == "cpu"))
        res[dev] = (formats.read_kernel(os.path.join(d, "kernel.tmp"))["weights"],
                    formats.read_kernel(os.path.join(d, "kernel.opt"))["weights"])
    for (w0c, w1c, w1g) in zip(res["cpu"][0], res["cpu"][1], res["gpu"][1]):
        dc, dg = w1c - w0c, w1g - w0c
        rel = np.linalg.norm(dc - dg) / (np.linalg.norm(dc) + 1e-30)
        assert rel < 0.08, rel


def test_run_nn_gpu(tmp_path):
    d = str(tmp_path)
    _data(os.path.join(d, "samples"), 20, 50, 4, True)
    formats.write_conf(os.path.join(d, "nn.conf"), name="t", type="SNN", seed=5, inputs=50, hiddens=[16], outputs=4,
                       train="BP", sample_dir="./samples", test_dir="./samples")
    out_g = _run([os.path.join(BIN, "run_nn"), "-vv", "nn.conf"], d)
    out_c = _run([os.path.join(BIN, "run_nn"), "-vv", "nn.conf"], d, cpu=True)
    assert out_g.count("[PASS]") == out_c.count("[PASS]")


@pytest.mark.parametrize("shape,dtype", [("fused", "bf16"), ("generic", "bf16"), ("generic", "f64")])
@pytest.mark.parametrize("dp_env", [{"HPNN_LOOPBACK_RANKS": "2"}, {"HPNN_LOOPBACK_RANKS": "3"},
                                    {"HPNN_FORCE_RCCL": "1"}])
def test_batched_data_parallel_matches_single(tmp_path, shape, dtype, dp_env):
    """native data-parallel path (csrc/gpu/gpu_engine.cpp train_dp): replicas each take a
    shard of every minibatch, gradients are summed (loopback: virtual replicas on one GPU;
    HPNN_FORCE_RCCL: a real 1-GPU RCCL communicator) -> same training as one replica."""
    if shape == "fused":
        dims = dict(inputs=784, hiddens=[128, 64], outputs=10, type="SNN")
    else:
        dims = dict(inputs=100, hiddens=[48], outputs=7, type="ANN")
    res = {}
    for tag, env in (("single", {}), ("dp", dp_env)):
        d = str(tmp_path / tag)
        _data(os.path.join(d, "samples"), 333, dims["inputs"], dims["outputs"], dims["type"] == "SNN")
        formats.write_conf(os.path.join(d, "nn.conf"), name="m", seed=9, train="BPM", sample_dir="./samples",
                           test_dir="./samples", mode="batched", batch=256, epochs=2, lr=0.05, dtype=dtype, **dims)
        out = _run([os.path.join(BIN, "train_nn"), "-vv", "nn.conf"], d, extra_env=env)
        assert ("data-parallel batched training" in out) == (tag == "dp"), out[-2000:]
        res[tag] = (formats.read_kernel(os.path.join(d, "kernel.tmp"))["weights"],
                    formats.read_kernel(os.path.join(d, "kernel.opt"))["weights"])
    for (w0, ws, wd) in zip(res["single"][0], res["single"][1], res["dp"][1]):
        ds, dd = ws - w0, wd - w0
        rel = np.linalg.norm(ds - dd) / (np.linalg.norm(ds) + 1e-30)
        # bf16: different batch shards round differently; f64: summation order only
        assert rel < (0.03 if dtype == "bf16" else 1e-11), rel


@pytest.mark.parametrize("dims,dtype", [((784, [128, 64], 10), "bf16"), ((40, [48], 6), "bf16"),
                                        ((40, [48], 6), "f64")])
def test_batched_gpu_exact_resume(tmp_path, dims, dtype):
    """GPU batched BPM: 2 epochs in one run == 1 epoch + state + 1 resumed epoch, bit for
    bit (FP32 master weights and momentum round-trip exactly through the FP64 state), with
    the HPNN_DEBUG serialised-launch mode and JSON metrics on."""
    n_in, hid, n_out = dims
    a, b = tmp_path / "a", tmp_path / "b"
    for d in (a, b):
        _data(str(d / "s"), 300, n_in, n_out, True, seed=4)
        formats.write_conf(str(d / "nn.conf"), name="r", type="SNN", seed=5, inputs=n_in, hiddens=hid,
                           outputs=n_out, train="BPM", sample_dir="./s", test_dir="./s", dtype=dtype)
    tn = os.path.join(BIN, "train_nn")
    env = {"HPNN_DEBUG": "1", "HPNN_METRICS": "m.jsonl"}
    _run([tn, "-b", "128", "-e", "2", "-r", "st.bin", "nn.conf"], str(a), extra_env=env)
    _run([tn, "-b", "128", "-e", "1", "-r", "st.bin", "nn.conf"], str(b), extra_env=env)
    out = _run([tn, "-vv", "-b", "128", "-e", "1", "-r", "st.bin", "nn.conf"], str(b), extra_env=env)
    assert "momentum restored" in out
    assert (a / "st.bin").read_bytes() == (b / "st.bin").read_bytes()
    assert (a / "kernel.opt").read_bytes() == (b / "kernel.opt").read_bytes()
    import json
    ep = [json.loads(x) for x in open(b / "m.jsonl")]
    assert [r["epoch"] for r in ep if r["event"] == "epoch"] == [1, 2]
    assert all(r["engine"] == "gpu" for r in ep if r["event"] == "epoch")


def test_batched_gpu_tn_update_matches_separate(tmp_path):
    """native batched engine: layers of 256x256 tiles with one gradient split take the
    weight-gradient GEMM with the optimizer step in its epilogue (hpnn_gemm_tn8_update);
    same training as the separate gradient + update kernels (HPNN_TN_UPD=0)"""
    res = {}
    for tag, env in (("fused", {}), ("separate", {"HPNN_TN_UPD": "0"})):
        d = str(tmp_path / tag)
        _data(os.path.join(d, "samples"), 256, 256, 256, False, seed=4)
        formats.write_conf(os.path.join(d, "nn.conf"), name="w", type="ANN", seed=13, inputs=256, hiddens=[256],
                           outputs=256, train="BPM", sample_dir="./samples", test_dir="./samples", mode="batched",
                           batch=256, epochs=3, lr=0.05, dtype="bf16")
        _run([os.path.join(BIN, "train_nn"), "-vv", "nn.conf"], d, extra_env=env)
        res[tag] = (formats.read_kernel(os.path.join(d, "kernel.tmp"))["weights"],
                    formats.read_kernel(os.path.join(d, "kernel.opt"))["weights"])
    for w0, wf, ws in zip(res["fused"][0], res["fused"][1], res["separate"][1]):
        df, ds = wf - w0, ws - w0
        assert np.linalg.norm(ds) > 0
        rel = np.linalg.norm(df - ds) / np.linalg.norm(ds)
        assert rel < 1e-3, rel


@pytest.mark.parametrize("net,train,dims,slots", [("SNN", "BPM", (120, [64, 40], 10), 2),
                                                  ("ANN", "BPM", (70, [48, 200, 33], 7), 2),
                                                  ("SNN", "BP", (300, [700], 40), 2)])
def test_online_device_spanning_matches_single(tmp_path, net, train, dims, slots):
    """The online engine with its cooperative grid spread over several slots (one per GPU
    with train_nn -G N; here HPNN_ONLINE_SLOTS virtual slots on the box's one GPU, each its
    own launch on its own stream with its own copy of W, exchanging through fine-grained
    memory at system scope) == the one-device engine and the FP64 CPU engine to 1e-9.
    (Two slots: the slots' launches must run concurrently, and on one device more
    streams than hardware queues (GPU_MAX_HW_QUEUES = 4) would serialise them.)
    Every slot owns the rows j with (j mod total workgroups) in its range; the host gathers
    each row from its owner when the kernel is dumped.
    "streams": train_nn -S 2 without the variable -- the reference's rows over n_gpu x
    n_streams (libhpnn.c:471-505); on ONE device it is a no-op (two slots there measured
    slower, profiles/r4/a_online_engine.jsonl), so it must match the one-slot run."""
    n_in, hid, n_out = dims
    runs = {"cpu": (True, None, []), "one": (False, None, []),
            "slots": (False, {"HPNN_ONLINE_SLOTS": str(slots)}, []), "streams": (False, None, ["-S", "2"])}
    for tag, (cpu, env, flags) in runs.items():
        d = str(tmp_path / tag)
        _data(os.path.join(d, "samples"), 3, n_in, n_out, net == "SNN", seed=7)
        formats.write_conf(os.path.join(d, "nn.conf"), name="t", type=net, seed=9, inputs=n_in, hiddens=hid,
                           outputs=n_out, train=train, sample_dir="./samples", test_dir="./samples", lr=0.01)
        out = _run([os.path.join(BIN, "train_nn"), "-vv"] + flags + ["nn.conf"], d, cpu=cpu, extra_env=env)
        assert out.count("TRAINING FILE") == 3
        # -S 2 on one device is a documented no-op (one slot); HPNN_ONLINE_SLOTS forces two
        assert ("rows over 2 slots" in out) == (tag == "slots"), out[-2000:]
    ks = {t: formats.read_kernel(str(tmp_path / t / "kernel.opt"))["weights"] for t in runs}
    for a, b, c, e in zip(ks["cpu"], ks["one"], ks["slots"], ks["streams"]):
        assert np.abs(c - b).max() < 1e-9, np.abs(c - b).max()
        assert np.abs(c - a).max() < 1e-9, np.abs(c - a).max()
        assert np.abs(e - b).max() < 1e-9, np.abs(e - b).max()


@pytest.mark.parametrize("dtype,ranks,dims", [("f64", 2, (100, [48, 37], 7)), ("f64", 3, (64, [50], 9)),
                                              ("f32", 2, (100, [48, 37], 7)), ("f64", 4, (30, [20, 11, 13], 5))])
def test_batched_tensor_parallel_matches_single(tmp_path, dtype, ranks, dims):
    """[parallel] tp (csrc/gpu/tp_engine.cpp): every hidden layer's rows sharded over the
    ranks (here HPNN_LOOPBACK_RANKS host threads on the box's one GPU, exchanging through a
    device staging buffer; RCCL on a multi-GPU node), activations all-gathered, partial
    deltas reduce-scattered with f' applied on the reduced rows, the output layer
    replicated -> the same training as one GPU: f64 to summation order (1e-12), f32 1e-5.
    Uneven shards (48 / 37 / 11 / 13 rows over 2-4 ranks) exercise the zero padding."""
    n_in, hid, n_out = dims
    res = {}
    for tag, env, par in (("single", {}, "dp"), ("tp", {"HPNN_LOOPBACK_RANKS": str(ranks)}, "tp")):
        d = str(tmp_path / tag)
        _data(os.path.join(d, "samples"), 300, n_in, n_out, True, seed=6)
        formats.write_conf(os.path.join(d, "nn.conf"), name="m", type="SNN", seed=9, inputs=n_in, hiddens=hid,
                           outputs=n_out, train="BPM", sample_dir="./samples", test_dir="./samples",
                           mode="batched", batch=128, epochs=2, lr=0.05, dtype=dtype, parallel=par)
        out = _run([os.path.join(BIN, "train_nn"), "-vv", "nn.conf"], d, extra_env=env)
        assert ("tensor-parallel batched training" in out) == (tag == "tp"), out[-2000:]
        res[tag] = (formats.read_kernel(os.path.join(d, "kernel.tmp"))["weights"],
                    formats.read_kernel(os.path.join(d, "kernel.opt"))["weights"])
    for (w0, ws, wt) in zip(res["single"][0], res["single"][1], res["tp"][1]):
        ds, dt = ws - w0, wt - w0
        rel = np.linalg.norm(ds - dt) / (np.linalg.norm(ds) + 1e-30)
        assert rel < (1e-12 if dtype == "f64" else 1e-5), rel


@pytest.mark.parametrize("dtype", ["f64", "bf16"])
def test_batched_tensor_parallel_rccl_graphs(tmp_path, dtype):
    """[parallel] tp over a real RCCL communicator (HPNN_FORCE_RCCL=1, one GPU): each epoch's
    launches, the collectives included, are captured once in a HIP graph and replayed (eager
    with HPNN_GRAPH=0) -- same weights either way, and the same as the loopback collectives."""
    res = {}
    for tag, env in (("graph", {"HPNN_FORCE_RCCL": "1"}), ("eager", {"HPNN_FORCE_RCCL": "1", "HPNN_GRAPH": "0"}),
                     ("loopback", {})):
        d = str(tmp_path / tag)
        _data(os.path.join(d, "samples"), 300, 100, 7, True, seed=6)
        formats.write_conf(os.path.join(d, "nn.conf"), name="m", type="SNN", seed=9, inputs=100, hiddens=[48, 37],
                           outputs=7, train="BPM", sample_dir="./samples", test_dir="./samples", mode="batched",
                           batch=128, epochs=3, lr=0.05, dtype=dtype, parallel="tp")
        out = _run([os.path.join(BIN, "train_nn"), "-vvv", "nn.conf"], d, extra_env=env)
        assert ("RCCL" in out) == (tag != "loopback"), out[-2000:]
        assert "not capturable" not in out, out[-2000:]
        res[tag] = formats.read_kernel(os.path.join(d, "kernel.opt"))["weights"]
    for a, b, c in zip(res["graph"], res["eager"], res["loopback"]):
        assert np.array_equal(a, b)
        assert np.abs(a - c).max() <= (1e-12 if dtype == "f64" else 1e-6) * max(1.0, np.abs(c).max())


@pytest.mark.parametrize("ranks,dims,batch", [(2, (100, [48, 37], 7), 128), (3, (64, [50], 9), 100),
                                               (4, (784, [128, 64], 10), 256)])
def test_batched_tensor_parallel_bf16(tmp_path, ranks, dims, batch):
    """[parallel] tp with [dtype] bf16 (tp_engine.cpp TpNetBf16): the row sharding on the BF16
    MFMA kernels, batch-major activations all-gathered in BF16 and block-permuted, partial
    deltas reduce-scattered in FP32 with f' fused into the BF16 cast.  P ranks == one rank of
    the same engine up to the FP32 summation order of the deltas (BF16 rounding flips: 1e-2),
    and both close to the data-parallel-free single-GPU batched engine (different kernels,
    3e-2).  batch 100: the batch padded to 128 with zero samples."""
    n_in, hid, n_out = dims
    res = {}
    for tag, env, par in (("single", {}, "dp"), ("tp1", {}, "tp"), ("tp", {"HPNN_LOOPBACK_RANKS": str(ranks)}, "tp")):
        d = str(tmp_path / tag)
        _data(os.path.join(d, "samples"), 300, n_in, n_out, True, seed=6)
        formats.write_conf(os.path.join(d, "nn.conf"), name="m", type="SNN", seed=9, inputs=n_in, hiddens=hid,
                           outputs=n_out, train="BPM", sample_dir="./samples", test_dir="./samples",
                           mode="batched", batch=batch, epochs=2, lr=0.05, dtype="bf16", parallel=par)
        out = _run([os.path.join(BIN, "train_nn"), "-vv", "nn.conf"], d, extra_env=env)
        assert ("tensor-parallel batched training" in out) == (tag != "single"), out[-2000:]
        if tag != "single":
            assert "bf16" in out
        res[tag] = (formats.read_kernel(os.path.join(d, "kernel.tmp"))["weights"],
                    formats.read_kernel(os.path.join(d, "kernel.opt"))["weights"])
    for (w0, ws, w1, wt) in zip(res["single"][0], res["single"][1], res["tp1"][1], res["tp"][1]):
        ds, d1, dt = ws - w0, w1 - w0, wt - w0
        assert np.linalg.norm(d1) > 0
        rel = np.linalg.norm(d1 - dt) / np.linalg.norm(d1)
        assert rel < 1e-2, rel
        rel = np.linalg.norm(ds - dt) / (np.linalg.norm(ds) + 1e-30)
        assert rel < 3e-2, rel


@pytest.mark.parametrize("dtype", ["bf16", "f64"])
def test_run_nn_sharded_evaluation_matches(tmp_path, dtype):
    """run_nn's batched GPU evaluation split into contiguous sample shards, one host thread
    each on its own (device, stream) (run_nn -G N -S M; here -S 2 on the box's one GPU, and
    HPNN_INFER_SHARDS=3 shards on new streams) == the unsplit evaluation, line for line."""
    d = str(tmp_path)
    _data(os.path.join(d, "samples"), 301, 60, 5, True, seed=3)
    formats.write_conf(os.path.join(d, "nn.conf"), name="t", type="SNN", seed=5, inputs=60, hiddens=[48, 32],
                       outputs=5, train="BP", sample_dir="./samples", test_dir="./samples", dtype=dtype)
    one = _run([os.path.join(BIN, "run_nn"), "-vvv", "nn.conf"], d)
    three = _run([os.path.join(BIN, "run_nn"), "-vvv", "nn.conf"], d, extra_env={"HPNN_INFER_SHARDS": "3"})
    assert "over 3 shards" in three
    streams = _run([os.path.join(BIN, "run_nn"), "-vvv", "-S", "2", "nn.conf"], d)  # -S: (GPU, stream) shards
    assert "over 2 (GPU, stream) shards" in streams
    import re
    # the per-class probabilities (10 digits) and the verdict of every file
    lines = lambda out: [x for x in out.splitlines() if "BEST CLASS" in x or re.match(r"^\s*\d+ \|", x)]  # noqa
    assert sum("BEST CLASS" in x for x in lines(one)) == 301
    assert lines(one) == lines(three) == lines(streams)
