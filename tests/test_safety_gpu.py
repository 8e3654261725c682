"""Runtime defences of the in-kernel hand-offs:

* residency guard: a fused G0 grid larger than the device holds at once (forced splits) takes
  the slab form instead of spinning to its 10 s timeout;
* 64-bit split-K tickets: launches whose tickets cross 2^32 still reduce every split;
* health readback: a hand-off that reports a timeout stops train_nn and bench.py;
* replica consistency: a replica whose weights drift makes bench.py exit 3 and train_nn stop.

Reference analogue: CHK_ERR after every launch (include/libhpnn/common.h:324-335) and the MPI
bail-out (src/ann.c:237-249)."""
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from hpnn_amd.models import MLP
from hpnn_amd.utils import formats

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TN = os.path.join(ROOT, "bin", "train_nn")
MNIST = [784, 128, 64, 10]


def _batch(m, seed=3):
    g = torch.Generator(device="cuda").manual_seed(seed)
    X = m.prepare_input(torch.randint(0, 256, (m.Bp, 784), device="cuda", generator=g, dtype=torch.uint8))
    lab = torch.randint(0, 10, (m.Bp,), device="cuda", generator=g, dtype=torch.int32)
    return X, lab


def test_forced_g0_splits_beyond_residency_take_slab_path(gpu):
    ref = MLP(MNIST, "SNN", batch=65536, momentum=True, fused="t")
    X, lab = _batch(ref)
    ref.train_step(X, labels=lab)
    torch.cuda.synchronize()
    # 64 splits x 10 tiles = 640 workgroups of the fused G0 > 256 resident (one per CU)
    m = MLP(MNIST, "SNN", batch=65536, momentum=True, fused="t", splits=[64, 0, 0])
    assert m.S[0] == 64
    m.train_step(X, labels=lab)  # first launch (module load) outside the timing
    torch.cuda.synchronize()
    m2 = MLP(MNIST, "SNN", batch=65536, momentum=True, fused="t", splits=[64, 0, 0])
    t0 = time.perf_counter()
    m2.train_step(X, labels=lab)
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 1.0, "a forced grid stalled (in-kernel wait timed out?)"
    assert m.healthy() and m2.healthy()
    for a, b in zip(ref.W32, m2.W32):
        torch.testing.assert_close(b, a, rtol=0, atol=2e-6)


def test_ticket_counters_past_2pow32(gpu):
    a = MLP(MNIST, "SNN", batch=16384, momentum=True, fused="t")
    b = MLP(MNIST, "SNN", batch=16384, momentum=True, fused="t")
    a.plan.g0_xcd = b.plan.g0_xcd = False  # the flat reduction's tile counters (the XCD level has its own)
    S = a.S[0]
    cnt = b.buf[("g0cnt", -1)].view(torch.int64)  # 64-bit tile counters, 32 words apart
    start = (2 ** 32 // S) * S  # the launches' tickets cross 2^32
    for tile in range(31):  # every tile counter the launch may use (HPNN_G0_MAX_TILES)
        cnt[16 * tile] = start
    X, lab = _batch(a)
    for _ in range(3):
        a.train_step(X, labels=lab)
        b.train_step(X, labels=lab)
    torch.cuda.synchronize()
    assert a.healthy() and b.healthy()
    assert int(cnt[0]) == start + 3 * S
    for wa, wb in zip(a.W32, b.W32):
        assert torch.equal(wa, wb)  # fixed-order reduction: bitwise equal


def test_digest_tracks_weights(gpu):
    a = MLP(MNIST, "SNN", batch=4096, momentum=True, fused="t")
    b = MLP(MNIST, "SNN", batch=4096, momentum=True, fused="t")
    assert a.weights_digest() == b.weights_digest()
    b.W32[1].view(-1)[7] += 2 ** -20
    b.refresh_bf16()
    assert a.weights_digest(2) != b.weights_digest(2)


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
              "LOCAL_WORLD_SIZE", "HPNN_FAULT"):
        e.pop(k, None)
    e.update({k: str(v) for k, v in kw.items()})
    return e


def _mnist_dir(tmp_path):
    _data(str(tmp_path / "s"), 600, 784, 10)
    formats.write_conf(str(tmp_path / "nn.conf"), name="f", type="SNN", seed=4, inputs=784, hiddens=[128, 64],
                       outputs=10, train="BPM", sample_dir="./s", test_dir="./s", dtype="bf16")


def test_train_nn_stops_on_handoff_timeout(gpu, tmp_path):
    _mnist_dir(tmp_path)
    flags = ["-v", "-b", "512", "-e", "3", "nn.conf"]
    ok = subprocess.run([TN] + flags, cwd=tmp_path, env=_env(), capture_output=True, text=True, timeout=300)
    assert ok.returncode == 0, ok.stdout[-2000:] + ok.stderr[-2000:]
    r = subprocess.run([TN] + flags, cwd=tmp_path, env=_env(HPNN_FAULT="handoff:1"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert "hand-off timed out" in r.stderr and "Training FAILED" in r.stderr, r.stderr[-2000:]


def test_train_nn_two_processes_stop_on_replica_mismatch(gpu, tmp_path):
    _mnist_dir(tmp_path)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    flags = ["-v", "-b", "512", "-e", "2", "nn.conf"]
    procs = [subprocess.Popen([TN] + flags, cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                              env=_env(RANK=r, WORLD_SIZE=2, LOCAL_RANK=0, LOCAL_WORLD_SIZE=2,
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                                       HPNN_BOOT_DIR=str(tmp_path / "boot"), HPNN_BOOT_TIMEOUT_S=60,
                                       HPNN_XAR_TIMEOUT_MS=3000, HPNN_FAULT="digest:1"))
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
    assert all(rc != 0 for rc, _, _ in outs), [o[-500:] + e[-500:] for _, o, e in outs]
    assert "replicas' weights differ" in outs[0][2], outs[0][2][-2000:]


def test_bench_exits_3_when_a_replica_drifts(gpu):
    env = _env(HPNN_BENCH_REHEARSE=1, HPNN_FAULT="weights:1")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--steps", "4", "--warmup", "2", "--batch", "4096", "--graph-steps", "2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert "replica weights differ after the timed steps" in r.stderr, r.stderr[-3000:]
    assert '"metric"' not in r.stdout
    assert r.returncode != 0
    assert "exitcode: 3" in r.stderr or "exit code: 3" in r.stderr or "exitcode  : 3" in r.stderr, r.stderr[-3000:]


def test_g0_role_order_permuted_bitwise(gpu):
    """the fused G0 launch (split-K tickets, fixed-order split sums, [G1 | G2] share, steps)
    gives bitwise the same weights whichever workgroup takes which (tile, split) role: the
    grid run in reversed and rotated block orders.  The XCD-aware role order is a speed
    assumption, never a correctness one."""
    runs = {}
    for perm in (0, 240, 1, 97):  # 240 workgroups: 240 = reversed, 1 / 97 = reversed + rotated
        m = MLP(MNIST, "SNN", batch=65536, momentum=True, fused="t")
        assert m.S[0] * 10 == 240 or m.S[0] * 5 == 240, m.S[0]
        m.plan.g0_perm = perm
        X, lab = _batch(m)
        for _ in range(2):
            m.train_step(X, labels=lab)
        torch.cuda.synchronize()
        assert m.healthy()
        runs[perm] = [t.clone() for t in list(m.W32) + list(m.V32) + list(m.Wb)]
        del m
    for perm in (240, 1, 97):
        for a, b in zip(runs[0], runs[perm]):
            assert torch.equal(a, b), perm


def test_bench_degrades_when_an_in_kernel_sum_is_wrong(gpu):
    """a cross-rank sum that arrives in time but is wrong (HPNN_FAULT=xsum:1: rank 1's first
    in-kernel exchange sums one element wrong) no longer kills the run: the replicas disagree
    after the first step, every rank leaves the xGMI exchange for the next one (RCCL, here
    torch.distributed: the ranks share one GPU), rank 0's weights are re-broadcast, the
    replicas agree again and the bench reports a number (reference: the P2P -> CMM -> EXP
    fallback chain, libhpnn.c:245-302)"""
    env = _env(HPNN_BENCH_REHEARSE=1, HPNN_REHEARSE_FUSED=1, HPNN_SPLITS="8,0,0", HPNN_FAULT="xsum:1",
               HPNN_XAR_TIMEOUT_MS=5000)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--steps", "4", "--warmup", "2", "--batch", "4096", "--graph-steps", "2", "--settle-ms", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "replica weights differ after the first step over xGMI; falling back" in r.stderr, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    import json
    out = json.loads(line[0])
    assert "xgmi" not in out["config"]["grad_allreduce"], out["config"]


def test_train_nn_leaves_xgmi_when_replicas_disagree(gpu, tmp_path):
    """train_dp_mp: a digest mismatch after the first (xGMI) epoch no longer stops the run at
    once -- the ranks leave the xGMI exchange, re-broadcast rank 0's weights and open RCCL
    (HPNN_FAULT=xdigest:1 makes the first digest look wrong on one rank).  Here both ranks
    share one GPU, where RCCL refuses to start, so the run then stops; on one GPU per rank it
    goes on over RCCL."""
    _mnist_dir(tmp_path)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    flags = ["-v", "-b", "512", "-e", "2", "nn.conf"]
    procs = [subprocess.Popen([TN] + flags, cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                              env=_env(RANK=r, WORLD_SIZE=2, LOCAL_RANK=0, LOCAL_WORLD_SIZE=2,
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                                       HPNN_BOOT_DIR=str(tmp_path / "boot"), HPNN_BOOT_TIMEOUT_S=60,
                                       HPNN_XAR_TIMEOUT_MS=3000, HPNN_FAULT="xdigest:1"))
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
    assert "falling back to RCCL from rank 0's weights" in outs[0][2], outs[0][2][-2000:]


def test_g0_xcd_local_level_bitwise(gpu):
    """the XCD-local first level of the fused G0's split-K reduction (plan.g0_xcd: members of a
    group combine through their XCD's L2, one write-through partial per (tile, group)): the
    same weights as the flat reduction up to FP32 summation order, and bitwise the same in a
    permuted block -> role order (the group's store form depends on where its members landed,
    read from the hardware XCC_ID; the sums keep one fixed order)"""
    runs = {}
    for key, xcd, perm in (("flat", False, 0), ("xcd", True, 0), ("xcd_perm", True, 97), ("xcd_rev", True, 240)):
        m = MLP(MNIST, "SNN", batch=65536, momentum=True, fused="t")
        m.plan.g0_xcd = xcd
        m.plan.g0_perm = perm
        X, lab = _batch(m)
        for _ in range(3):
            m.train_step(X, labels=lab)
        torch.cuda.synchronize()
        assert m.healthy()
        runs[key] = [t.clone() for t in list(m.W32) + list(m.V32)]
        del m
    for k in ("xcd_perm", "xcd_rev"):
        for a, b in zip(runs["xcd"], runs[k]):
            assert torch.equal(a, b), k
    for a, b in zip(runs["xcd"], runs["flat"]):
        torch.testing.assert_close(a, b, rtol=0, atol=2e-6)
