"""debug: mode x with a fragment-major copy: fused G0 (gradient-out and step) vs unfused"""
import sys
import torch
sys.path.insert(0, ".")
from hpnn_amd import ops
from hpnn_amd.models import MLP

for B in (16384, 8192):
    res = {}
    for fused in (True, False):
        torch.manual_seed(9)
        m = MLP([784, 128, 64, 10], "SNN", batch=B, seed=3, momentum=True, fused="x")
        m.plan.g0_fused = fused
        X = m.prepare_input(torch.rand(B, 784))
        X.hpnn_fm = ops.to_fragment_major(X)
        lab = torch.randint(0, 10, (B,), dtype=torch.int32, device="cuda",
                            generator=torch.Generator(device="cuda").manual_seed(1))
        segs = m.grads_slabs(X, labels=lab)
        torch.cuda.synchronize()
        if fused:
            g = m.grad_flat.clone()
        else:
            parts = []
            for addr, stride, cnt, n in segs:
                base = [t for t in (m.slab[0], m.midtmp) if t.data_ptr() == addr][0].reshape(-1)
                parts.append(torch.stack([base[s * stride:s * stride + n] for s in range(cnt)]).sum(0))
            g = torch.cat(parts)[:m.grad_flat.numel()]
        W0 = [w.clone() for w in m.W32]
        m.train_step(X, labels=lab, lr=0.05, alpha=0.2)
        torch.cuda.synchronize()
        res[fused] = (g, [m.W32[l] - W0[l] for l in range(3)], m.S[0], m.plan.health(torch.cuda.current_stream().cuda_stream))
    (ga, da, S, h), (gb, db, _, _) = res[True], res[False]
    print("B", B, "S0", S, "health", h, "segs fused", flush=True)
    print(f"  grad diff G0 {(ga[:102400] - gb[:102400]).abs().max().item():.3e} scale {gb[:102400].abs().max().item():.3e}"
          f"  G12 {(ga[102400:] - gb[102400:]).abs().max().item():.3e}")
    for l in range(3):
        print(f"  step dW{l} diff {(da[l] - db[l]).abs().max().item():.3e} scale {db[l].abs().max().item():.3e}")
