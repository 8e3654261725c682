"""FP64 / FP32 batched GPU engine ([dtype] f64 | f32, csrc/gpu/kernels_fp.hip): the
reference's precision on the FP64 / FP32 MFMA.

Kernel numerics against plain PyTorch FP64 / FP32 references of the same ops, and whole
training runs of train_nn (batched mode) against the FP64 CPU batched oracle
(csrc/cpu/cpu_batched.cpp): <= 1e-12 relative weight change for f64, <= 1e-5 for f32;
run_nn's batched GPU evaluation gives the same PASS/FAIL lines as the CPU engine."""
import os
import subprocess

import numpy as np
import pytest
import torch

from hpnn_amd._lib import native
from hpnn_amd.utils import formats

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _bip(x):
    return 2.0 / (1.0 + torch.exp(-x)) - 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float64, torch.float32])
@pytest.mark.parametrize("M,N,K,ta,tb,epi", [(300, 70, 130, 0, 0, 1), (257, 33, 65, 0, 1, 2), (40, 90, 1000, 1, 1, 0),
                                             (128, 64, 64, 0, 0, 0),
                                             # >= 256 tiles of 128 x 128: the large-GEMM kernel; odd
                                             # strides (scalar loads) and edges, every operand layout
                                             (2085, 2053, 303, 0, 0, 1), (2048, 2048, 512, 1, 1, 0),
                                             (2200, 2100, 334, 1, 0, 2), (2304, 2176, 100, 0, 1, 1)])
def test_gemm_fp_matches_torch(gpu, dt, M, N, K, ta, tb, epi):
    torch.manual_seed(M + N + K)
    A = torch.randn(K, M, dtype=dt, device="cuda") if ta else torch.randn(M, K, dtype=dt, device="cuda")
    B = torch.randn(K, N, dtype=dt, device="cuda") if tb else torch.randn(N, K, dtype=dt, device="cuda")
    aux = torch.rand(M, N, dtype=dt, device="cuda") * 2 - 1
    f64 = int(dt == torch.float64)
    splits = 3 if epi == 0 else 1
    C = torch.zeros(splits, M, N, dtype=dt, device="cuda")
    S = native().gemm_fp(f64, A.data_ptr(), A.stride(0), ta, B.data_ptr(), B.stride(0), tb, C.data_ptr(), N,
                         aux.data_ptr(), N, M, N, K, epi, splits, M * N, _stream())
    torch.cuda.synchronize()
    a = (A.t() if ta else A).double()
    b = (B if tb else B.t()).double()
    ref = a @ b
    if epi == 1:
        ref = _bip(ref)
    elif epi == 2:
        ref = ref * (-0.5 * (aux.double() ** 2 - 1))
    got = C[:S].sum(0).double()
    tol = 1e-12 if f64 else 2e-5
    assert (got - ref).abs().max().item() <= tol * (ref.abs().max().item() + 1)


@pytest.mark.gpu
@pytest.mark.parametrize("net", [0, 1, 2])
def test_output_fp_matches_reference(gpu, net):
    torch.manual_seed(net)
    B, n_out = 333, 37
    Z = torch.randn(B, n_out, dtype=torch.float64, device="cuda") * 3
    T = torch.zeros(B, n_out, dtype=torch.float64, device="cuda") - (0.0 if net == 2 else 1.0)
    lab = torch.randint(0, n_out, (B,), device="cuda")
    T[torch.arange(B), lab] = 1.0
    D = torch.empty_like(Z)
    O = torch.empty_like(Z)
    guess = torch.empty(B, dtype=torch.int32, device="cuda")
    stats = torch.zeros(64, 16, device="cuda")
    native().output_fp(1, Z.data_ptr(), n_out, T.data_ptr(), n_out, D.data_ptr(), n_out, O.data_ptr(), n_out,
                       guess.data_ptr(), stats[0, 0:1].data_ptr(), stats[0, 1:2].data_ptr(), B, B - 5, n_out, net,
                       _stream())
    torch.cuda.synchronize()
    if net == 2:  # reference form e^{z-1} / (TINY + sum e^{z-1})
        e = torch.exp(Z - 1)
        o = e / (1e-14 + e.sum(1, keepdim=True))
        d = T - o
    elif net == 0:
        o = _bip(Z)
        d = (T - o) * (-0.5 * (o * o - 1))
    else:
        o = Z
        d = T - o
    assert (O - o).abs().max().item() < 1e-14
    assert (D[:B - 5] - d[:B - 5]).abs().max().item() < 1e-14
    assert torch.count_nonzero(D[B - 5:]) == 0
    assert torch.equal(guess.long(), o.argmax(1))
    hits = int(stats[:, 1].contiguous().view(torch.int32).sum())
    assert hits == int((o.argmax(1) == lab)[:B - 5].sum())


def _data(d, n, n_in, n_out, snn, seed=1):
    rng = np.random.default_rng(seed)
    os.makedirs(d, exist_ok=True)
    for i in range(n):
        x = rng.uniform(-1, 1, n_in)
        t = np.full(n_out, 0.0 if snn else -1.0)
        t[int(rng.integers(n_out))] = 1.0
        formats.write_sample(os.path.join(d, f"s{i:04d}.txt"), x, t)


def _run(cmd, cwd, cpu=False, extra_env=None):
    env = dict(os.environ)
    env.pop("HPNN_FORCE_CPU", None)
    if cpu:
        env["HPNN_FORCE_CPU"] = "1"
    env.update(extra_env or {})
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.gpu
# f32: FP32 rounding of gradient sums with cancellation over 128 samples x 784 inputs;
# measured 1.6e-5 (SNN) / 4.2e-5 (ANN) relative against the FP64 oracle
@pytest.mark.parametrize("dtype,tol", [("f64", 1e-12), ("f32", 1e-4)])
@pytest.mark.parametrize("net,train,dims", [("SNN", "BPM", (784, [128, 64], 10)), ("ANN", "BP", (40, [48, 20], 6)),
                                            ("LNN", "BPM", (33, [17], 5))])
def test_train_nn_fp_matches_cpu_oracle(tmp_path, gpu, dtype, tol, net, train, dims):
    n_in, hid, n_out = dims
    res = {}
    for dev in ("cpu", "gpu"):
        d = str(tmp_path / dev)
        _data(os.path.join(d, "samples"), 300, n_in, n_out, net == "SNN")
        formats.write_conf(os.path.join(d, "nn.conf"), name="fp", type=net, seed=9, inputs=n_in, hiddens=hid,
                           outputs=n_out, train=train, sample_dir="./samples", test_dir="./samples", mode="batched",
                           batch=128, epochs=2, lr=0.05, dtype=dtype)
        out = _run([os.path.join(BIN, "train_nn"), "-vv", "nn.conf"], d, cpu=(dev == "cpu"),
                   extra_env={"HPNN_KERNEL_EXACT": "1"})
        if dev == "gpu":
            assert f"batched GPU training: {dtype}" in out, out[-2000:]
        res[dev] = (formats.read_kernel(os.path.join(d, "kernel.tmp"))["weights"],
                    formats.read_kernel(os.path.join(d, "kernel.opt"))["weights"])
    for w0, wc, wg in zip(res["cpu"][0], res["cpu"][1], res["gpu"][1]):
        dc, dg = wc - w0, wg - w0
        rel = np.linalg.norm(dc - dg) / (np.linalg.norm(dc) + 1e-300)
        assert rel <= tol, rel  # (kernel files written with %.17g: HPNN_KERNEL_EXACT)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["f64", "bf16"])
def test_run_nn_batched_gpu_matches_cpu(tmp_path, gpu, dtype):
    d = str(tmp_path)
    _data(os.path.join(d, "samples"), 1000, 60, 7, True, seed=3)
    formats.write_conf(os.path.join(d, "nn.conf"), name="t", type="SNN", seed=5, inputs=60, hiddens=[32], outputs=7,
                       train="BP", sample_dir="./samples", test_dir="./samples", dtype=dtype)
    out_g = _run([os.path.join(BIN, "run_nn"), "-vv", "nn.conf"], d)
    out_c = _run([os.path.join(BIN, "run_nn"), "-vv", "nn.conf"], d, cpu=True)
    lines_g = [ln for ln in out_g.splitlines() if "TESTING FILE" in ln]
    lines_c = [ln for ln in out_c.splitlines() if "TESTING FILE" in ln]
    assert len(lines_g) == len(lines_c) == 1000
    if dtype == "f64":  # same file order, same verdict per file
        assert [ln.split("BEST")[0] + ln.split("]")[-2][-6:] for ln in lines_g] == \
               [ln.split("BEST")[0] + ln.split("]")[-2][-6:] for ln in lines_c]
        assert out_g.count("[PASS]") == out_c.count("[PASS]")
    else:
        assert abs(out_g.count("[PASS]") - out_c.count("[PASS]")) <= 10
