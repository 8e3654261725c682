"""debug: fused G0 (gradient-out) published partial slabs vs the unfused kernel's slabs, and the
reduced G0 vs the sum of either"""
import sys
import torch
sys.path.insert(0, ".")
from hpnn_amd.models import MLP

for u8, Bp in ((True, 24576), (False, 8192)):
    res = {}
    for fused in (True, False):
        torch.manual_seed(5)
        m = MLP([784, 128, 64, 10], "SNN", batch=Bp, momentum=True, seed=5, fused="t")
        X = torch.randint(0, 256, (Bp, 784), dtype=torch.uint8) if u8 else torch.rand(Bp, 784) - 0.5
        m.plan.g0_fused = fused
        Xg = m.prepare_input(X.cuda())
        lab = torch.randint(0, 10, (Bp,), dtype=torch.int32, device="cuda",
                            generator=torch.Generator(device="cuda").manual_seed(9))
        m.slab[0].fill_(float("nan"))
        segs = m.grads_slabs(Xg, labels=lab)
        torch.cuda.synchronize()
        res[fused] = (m.slab[0].clone(), m.grad_flat[:128 * 800].clone().view(128, 800))
        print("u8", u8, "Bp", Bp, "fused", fused, "slab shape", tuple(m.slab[0].shape), "S", m.S[0], flush=True)
    sf, gf = res[True]
    ss, _ = res[False]
    S = ss.shape[0]
    for s in range(S):
        d = (sf[s] - ss[s]).abs()
        nan = torch.isnan(sf[s]).sum().item()
        if s < 4 or s > S - 3 or nan or d.max().item() > 1e-3:
            # where (rows/cols) the differences sit
            bad = (d > 1e-4) | torch.isnan(d)
            rows = bad.any(1).nonzero().flatten().tolist()
            cols = bad.any(0).nonzero().flatten().tolist()
            print(f"  split {s}: max diff {d.max().item():.3e} nan {nan} bad rows {rows[:8]}..{len(rows)} "
                  f"cols {cols[:8]}..{len(cols)}")
    ref = ss.sum(0)
    print(f"  G0 fused vs sum(sep slabs) {(gf - ref).abs().max().item():.3e}; "
          f"sum(fused slabs) vs sep {(sf.sum(0) - ref).abs().max().item():.3e}", flush=True)
