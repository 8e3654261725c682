"""LDS-DMA staged first-layer gradient (kernels_g0.hip fm_partial_lds, HPNN_G0_LDS=1): the
split slabs against the PyTorch reference (8-bit and BF16 H), and the fused step (in-kernel
split reduction + every layer's step) against the direct-load kernel's training, in a child
process (the switch is read once per process)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, torch
sys.path.insert(0, sys.argv[1])
from hpnn_amd import ops
from hpnn_amd.models import MLP
torch.manual_seed(0)
for u8 in (True, False):
    Bt, N, M, S = 4096, 128, 800, 8
    D = (torch.rand(Bt, N, device="cuda") - 0.5).bfloat16()
    H = torch.randint(0, 256, (Bt, M), dtype=torch.uint8, device="cuda") if u8 else (torch.rand(Bt, M, device="cuda") - 0.5).bfloat16()
    sc = 1.0 / 255 if u8 else 1.0
    slab = ops.gemm_fm_direct(ops.to_fragment_major(D), ops.to_fragment_major(H), N, M, splits=S, hscale=sc)
    torch.cuda.synchronize()
    ref = ops.ref_gemm_tn(D, H.bfloat16()) * sc  # 8-bit: exact integers, scale on the sums
    got = slab.sum(0)
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-3, ("slabs", u8, err)
    for s_, (a, b) in enumerate(ops.split_rows(Bt, S)):
        r = ops.ref_gemm_tn(D[a:b], H[a:b].bfloat16()) * sc
        e = ((slab[s_] - r).abs().max() / r.abs().max()).item()
        assert e < 2e-3, ("split", s_, e)
# fused step (two launches) with the LDS-staged G0 vs the per-layer path
B = 8192
X = torch.randint(0, 256, (B, 784), dtype=torch.uint8)
lab = torch.randint(0, 10, (B,), dtype=torch.int32, device="cuda")
mt = MLP([784, 128, 64, 10], "SNN", batch=B, momentum=True, seed=3, fused="t")
ml = MLP([784, 128, 64, 10], "SNN", batch=B, momentum=True, seed=3, fused=False)
Xt, Xl = mt.prepare_input(X.cuda()), ml.prepare_input(X.cuda())
for _ in range(3):
    mt.train_step(Xt, labels=lab, lr=0.05)
    ml.train_step(Xl, labels=lab, lr=0.05)
torch.cuda.synchronize()
assert mt.plan.health(torch.cuda.current_stream().cuda_stream) == 0
for a, b in zip(mt.host_weights(), ml.host_weights()):
    assert (a - b).abs().max().item() < 2e-3 * (b.abs().max().item() + 1e-3), (a - b).abs().max().item()
print("ok")
'''


@pytest.mark.gpu
def test_g0_lds_staged_matches_reference(gpu):
    env = dict(os.environ, HPNN_G0_LDS="1")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
