"""debug: fused G0 gradient-out vs slab sums, per column / row pattern of the difference"""
import sys
import torch
sys.path.insert(0, ".")
from hpnn_amd.models import MLP

for u8 in (True, False):
    for Bp in (24576, 8192):
        res = {}
        for fused in (True, False):
            torch.manual_seed(5)
            m = MLP([784, 128, 64, 10], "SNN", batch=Bp, momentum=True, seed=5, fused="t")
            X = torch.randint(0, 256, (Bp, 784), dtype=torch.uint8) if u8 else torch.rand(Bp, 784) - 0.5
            m.plan.g0_fused = fused
            Xg = m.prepare_input(X.cuda())
            lab = torch.randint(0, 10, (Bp,), dtype=torch.int32, device="cuda",
                                generator=torch.Generator(device="cuda").manual_seed(9))
            segs = m.grads_slabs(Xg, labels=lab)
            torch.cuda.synchronize()
            if fused:
                g = m.grad_flat.clone()
            else:
                parts = []
                for addr, stride, cnt, n in segs:
                    base = [t for t in (m.slab[0], m.midtmp) if t.data_ptr() == addr][0].reshape(-1)
                    parts.append(torch.stack([base[s * stride:s * stride + n] for s in range(cnt)]).sum(0))
                g = torch.cat(parts)[:m.grad_flat.numel()]
            res[fused] = g
            print("u8", u8, "Bp", Bp, "fused", fused, "segs", [(s[1], s[2], s[3]) for s in segs], "S0", m.S[0],
                  "health", m.plan.health(torch.cuda.current_stream().cuda_stream), flush=True)
        a, b = res[True], res[False]
        G0a, G0b = a[:128 * 800].view(128, 800), b[:128 * 800].view(128, 800)
        d = (G0a - G0b).abs()
        sc = G0b.abs().max().item()
        print(f"  G0 max diff {d.max().item():.3e} (scale {sc:.3e})")
        col = d.max(0).values
        bad = (col > 1e-4 * sc).nonzero().flatten().tolist()
        print("  bad cols", bad[:40], "n", len(bad))
        row = d.max(1).values
        badr = (row > 1e-4 * sc).nonzero().flatten().tolist()
        print("  bad rows", badr[:40], "n", len(badr))
        r = (a[128 * 800:] - b[128 * 800:]).abs()
        print(f"  G12 max diff {r.max().item():.3e} (scale {b[128 * 800:].abs().max().item():.3e})", flush=True)
