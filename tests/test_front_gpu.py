"""The role-split MLP front kernel (kernels_mlp3f.hip, selected with HPNN_FRONT=f) against
the per-layer path, the default fused kernel, and itself (bitwise repeatability).  The
kernel choice is read once per process, so every case runs in a child process with
HPNN_FRONT set explicitly."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, torch
sys.path.insert(0, ROOT)
from hpnn_amd.models import MLP
net_type, B, n_valid, n_out, dense = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] == "1"
torch.manual_seed(1)
sizes = [784, 128, 64, n_out]
mf = MLP(sizes, net_type, batch=B, momentum=True, seed=5, fused="x")
ml = MLP(sizes, net_type, batch=B, momentum=True, seed=5, fused=False)
X = mf.prepare_input(torch.rand(mf.Bp, 784))
kw = {}
if dense:
    lo = 0.0 if net_type == "SNN" else -1.0
    T = torch.full((mf.Bp, n_out), lo, device="cuda")
    T[torch.arange(mf.Bp), torch.randint(0, n_out, (mf.Bp,))] = 1.0
    kw["T"] = T
else:
    kw["labels"] = torch.randint(0, n_out, (mf.Bp,), dtype=torch.int32).cuda()
for _ in range(3):
    mf.train_step(X, n_valid=n_valid, lr=0.05, **kw)
    ml.train_step(X, n_valid=n_valid, lr=0.05, **kw)
torch.cuda.synchronize()
for a, b in zip(mf.host_weights(), ml.host_weights()):
    err = (a - b).abs().max().item()
    assert err < 2e-3 * (b.abs().max().item() + 1e-3), err
la, ca = mf.read_stats()
lb, cb = ml.read_stats()
assert abs(la - lb) <= 2e-2 * abs(lb), (la, lb)
assert abs(ca - cb) <= max(2, 0.01 * n_valid), (ca, cb)
assert torch.equal(mf.D[0][n_valid:], torch.zeros_like(mf.D[0][n_valid:]))
# bitwise repeatable: the same state and batch give the same weights
m2 = MLP(sizes, net_type, batch=B, momentum=True, seed=5, fused="x")
m3 = MLP(sizes, net_type, batch=B, momentum=True, seed=5, fused="x")
for m in (m2, m3):
    m.train_step(X, n_valid=n_valid, lr=0.05, **kw)
torch.cuda.synchronize()
assert all(torch.equal(a, b) for a, b in zip(m2.W32, m3.W32))
print("OK")
'''.replace("ROOT", repr(ROOT))


def _run(front, *args):
    env = {k: v for k, v in os.environ.items() if k not in ("HPNN_FRONT", "HPNN_FZ_MODE")}
    env["HPNN_FRONT"] = front
    r = subprocess.run([sys.executable, "-c", CHILD, *map(str, args)], env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("net_type,B,n_valid,n_out,dense", [
    ("SNN", 65536, 65536, 10, 0),   # the benchmark shape: 8 tiles per workgroup
    ("SNN", 16384, 16000, 10, 0),   # 2 tiles per workgroup, padded rows
    ("SNN", 640, 600, 10, 0),       # one tile per workgroup
    ("ANN", 4096, 4096, 20, 0),     # two output tiles
    ("LNN", 2048, 2000, 10, 0),
    ("SNN", 2048, 2048, 20, 1),     # dense targets
    ("ANN", 3072, 3072, 10, 1),
])
def test_role_split_front_matches_layerwise(gpu, net_type, B, n_valid, n_out, dense):
    _run("f", net_type, B, n_valid, n_out, dense)
