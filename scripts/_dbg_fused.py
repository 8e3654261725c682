import torch, sys, os
sys.path.insert(0, os.getcwd())
from hpnn_amd import ops
from hpnn_amd.models import MLP
torch.manual_seed(3)
for B in (256, 8192, 65536):
    m = MLP([784, 128, 64, 10], "SNN", batch=B, seed=4, fused="x")
    print("W0f ok", torch.equal(m.W0f, ops.frag_major(m.Wb[0])))
    X = m.prepare_input(torch.rand(B, 784))
    lab = torch.randint(0, 10, (B,), dtype=torch.int32, device="cuda")
    m.reset_stats()
    m._fused_front(X, lab, None, B)
    torch.cuda.synchronize()
    slab = torch.zeros(1, ops.MLP3_SLAB)
    D1 = torch.empty(B, 128, dtype=torch.bfloat16)
    st = torch.zeros(64, 16)
    ops.mlp3_fused(X.cpu(), m.Wb[0].cpu(), None, m.Wb[1].cpu(), m.Wb[2].cpu(), D1, slab, 10, ops.TYPE_SNN,
                   labels=lab.cpu(), n_valid=B, loss_acc=st[0, 0:1], correct=st[0, 1:2])
    g = m.D[0].cpu().float(); r = D1.float()
    err = (g - r).abs()
    print("B", B, "D1 max err", err.max().item(), "ref max", r.abs().max().item(), "rows bad", (err.max(1).values > 1e-2 * r.abs().max()).nonzero().flatten()[:20].tolist())
    gs = m.midslab.sum(0).cpu()
    print("G1 err", (gs[:8192] - slab[0, :8192]).abs().max().item(), "ref", slab[0, :8192].abs().max().item())
    print("G2 err", (gs[8192:] - slab[0, 8192:]).abs().max().item(), "ref", slab[0, 8192:].abs().max().item())
    print("stats", m.read_stats(), st[0, 0].item(), int(st[0, 1].view(torch.int32)))
