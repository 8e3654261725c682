"""Row-sharded tensor parallelism -- the reference's model-parallel scheme, on RCCL.

The reference splits every layer's neuron rows across MPI ranks / GPU streams, computes
its slice of each layer, and re-assembles the activations, deltas AND the full weight
matrices with all-gathers after every layer and every update (ann.c:912-1860,
cuda_ann.cu:533-2898).  Here, per hidden layer l with rows R_r owned by rank r (the same
scheme as the C engine's [parallel] tp, csrc/gpu/tp_engine.cpp TpNetBf16):

  forward   Hl_l = f(H_{l-1} . W_l[R_r]^T)                gemm_nt, ACT epilogue (local)
            stage = all_gather(Hl_l)  [P, B, n_l]          BF16
            H_l = block_permute(stage) [B, P n_l]          one kernel pass
  output    replicated (narrow): Z, softmax / loss / delta_L identical on every rank
  backward  Dl_{L-2} = f'(Hl) * (delta_L . W_L[:, R_r])      gemm_nt, DACT epilogue
            part[q] = Dl_l . W_l[R_q rows of layer l-1]^T    P gemm_nt, FP32 out
            Dl_{l-1} = bf16(f'(Hl_{l-1}) * reduce_scatter(part))  dact_cast kernel
  gradient  G_l[R_r] = Dl_l^T . H_{l-1}                     gemm_tn, split-K (local)
  update    every layer's local rows in one sgd_update_multi launch

so weights are never all-gathered (the reference moved N_l x M_l weights per layer per
step; this moves B x n_l BF16 activations and B x n_{l-1} FP32 partial deltas per rank).
Intended for layers too wide for one GPU's memory budget; the headline benchmark uses data
parallelism.  Every step runs on the gfx950 kernels (hpnn_amd.ops); CPU tensors run the ops'
PyTorch emulation (tests/test_tp_cpu.py).
"""
import torch
import torch.distributed as dist

from .. import ops
from .._lib import native
from ..models.mlp import TYPES, reference_init, fast_init


class TensorParallelMLP:
    def __init__(self, sizes, net_type="SNN", batch=256, device="cuda", momentum=False, seed=10958, group=None,
                 init="reference"):
        self.group = group
        self.P = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.sizes = list(sizes)
        self.L = len(sizes) - 1
        self.type = TYPES[net_type]
        self.device = torch.device(device)
        self.Bp = ops.pad_to(batch, 128)
        self.momentum = momentum
        P, L = self.P, self.L
        # hidden rows padded so each rank holds a multiple of 32; the output layer replicated
        self.Nr = [ops.pad_to(-(-sizes[l + 1] // P), 32) for l in range(L - 1)] + [ops.pad_to(sizes[-1], 32)]
        self.Np = [P * n for n in self.Nr[:-1]] + [self.Nr[-1]]
        self.Kp = [ops.pad_to(sizes[0], 32)] + self.Np[:-1]
        full = reference_init(sizes, seed) if init == "reference" else fast_init(sizes, seed)
        dev = self.device
        self.W32, self.V32, self.Wb, self.Wt, self.S = [], [], [], [], []
        for l in range(L):
            w = torch.zeros(self.Np[l], self.Kp[l], dtype=torch.float32)
            w[:sizes[l + 1], :sizes[l]] = full[l].float()
            r0 = self.rank * self.Nr[l] if l < L - 1 else 0
            wl = w[r0:r0 + self.Nr[l]].contiguous().to(dev)
            self.W32.append(wl)
            self.V32.append(torch.zeros_like(wl) if momentum else None)
            self.Wb.append(torch.empty_like(wl, dtype=torch.bfloat16))
            self.Wt.append(torch.empty(self.Kp[l], self.Nr[l], dtype=torch.bfloat16, device=dev))
            ops.cast_weights(self.W32[l], self.Wb[l], self.Wt[l])
            self.S.append(1 if dev.type == "cpu" else native().BPlan.pick_splits(self.Nr[l], self.Kp[l], self.Bp))
        bf = dict(dtype=torch.bfloat16, device=dev)
        self.Hl = [torch.empty(self.Bp, self.Nr[l], **bf) for l in range(L - 1)]      # local rows
        self.H = [torch.empty(self.Bp, self.Np[l], **bf) if P > 1 else self.Hl[l] for l in range(L - 1)]
        self.stage = [torch.empty(P, self.Bp, self.Nr[l], **bf) for l in range(L - 1)] if P > 1 else []
        self.Dl = [torch.empty(self.Bp, self.Nr[l], **bf) for l in range(L)]
        self.part = [None] + [torch.empty(P, self.Bp, self.Nr[l - 1], dtype=torch.float32, device=dev)
                              for l in range(1, L - 1)]
        self.dred = [None] + [torch.empty(self.Bp, self.Nr[l - 1], dtype=torch.float32, device=dev) if P > 1 else None
                              for l in range(1, L - 1)]
        self.G = [torch.empty(self.S[l], self.Nr[l], self.Kp[l], dtype=torch.float32, device=dev) for l in range(L)]
        self.Z = torch.empty(self.Bp, self.Nr[-1], dtype=torch.float32, device=dev)
        self.stats = torch.zeros(64, 16, dtype=torch.float32, device=dev)

    # RCCL (backend "nccl"): the tensor collectives in place.  gloo (CPU tests, or two ranks
    # sharing one GPU in tests/test_tp_gpu.py): through host copies; gloo has no
    # reduce-scatter, so the sum is all-reduced in rank order and this rank's block kept.
    def _nccl(self):
        return dist.get_backend(self.group) == "nccl"

    def _ag(self, out, inp):
        """out [P, *inp.shape] <- every rank's inp"""
        if self._nccl():
            dist.all_gather_into_tensor(out.view(-1, *inp.shape[1:]), inp, group=self.group)
            return
        parts = [torch.empty(inp.shape, dtype=inp.dtype) for _ in range(self.P)]
        dist.all_gather(parts, inp.cpu(), group=self.group)
        out.copy_(torch.stack(parts))

    def _rs(self, out, inp):
        """out <- sum over ranks of their inp[rank] (inp [P, *out.shape])"""
        if self._nccl():
            dist.reduce_scatter_tensor(out, inp.view(-1, *out.shape[1:]), group=self.group)
            return
        t = inp.cpu()
        dist.all_reduce(t, group=self.group)
        out.copy_(t[self.rank])

    def train_step(self, X, labels=None, T=None, n_valid=None, lr=0.01, alpha=0.2):
        n_valid = self.Bp if n_valid is None else n_valid
        L, P = self.L, self.P
        for l in range(L - 1):
            ops.gemm_nt(X if l == 0 else self.H[l - 1], self.Wb[l], ops.EPI_ACT, out=self.Hl[l])
            if P > 1:
                self._ag(self.stage[l], self.Hl[l])
                ops.block_permute(self.stage[l], self.H[l])
        Ho = X if L == 1 else self.H[L - 2]
        ops.gemm_nt(Ho, self.Wb[-1], ops.EPI_NONE, out_f32=True, out=self.Z)
        t_hi, t_lo = (1.0, 0.0) if self.type == ops.TYPE_SNN else (1.0, -1.0)
        ops.output_delta(self.Z, self.sizes[-1], self.type, self.Dl[-1], labels=labels, T=T, t_hi=t_hi, t_lo=t_lo,
                         n_valid=n_valid, loss_acc=self.stats[0, 0:1], correct=self.stats[0, 1:2])
        ops.gemm_tn(self.Dl[-1], Ho, splits=self.S[-1], out=self.G[-1])
        if L >= 2:
            h, r0 = L - 2, self.rank * self.Nr[L - 2]
            ops.gemm_nt(self.Dl[-1], self.Wt[-1][r0:r0 + self.Nr[h]], ops.EPI_DACT, aux=self.Hl[h], out=self.Dl[h])
        for l in range(L - 2, -1, -1):
            ops.gemm_tn(self.Dl[l], X if l == 0 else self.H[l - 1], splits=self.S[l], out=self.G[l])
            if l > 0:
                m = self.Nr[l - 1]
                for q in range(P):
                    ops.gemm_nt(self.Dl[l], self.Wt[l][q * m:(q + 1) * m], ops.EPI_NONE, out_f32=True,
                                out=self.part[l][q])
                red = self.part[l][0]
                if P > 1:
                    self._rs(self.dred[l], self.part[l])
                    red = self.dred[l]
                ops.dact_cast(self.Dl[l - 1], red, self.Hl[l - 1])
        layers = [(self.W32[l], self.V32[l], self.G[l], self.Wb[l], self.Wt[l], None) for l in range(L)]
        for i in range(0, L, 8):
            ops.sgd_update_multi(layers[i:i + 8], lr, alpha, 1.0 / n_valid, self.momentum)

    def full_weights(self):
        """gather the row shards (FP64 host, unpadded) -- checkpointing / tests."""
        out = []
        for l in range(self.L):
            w = self.W32[l]
            if self.P > 1 and l < self.L - 1:
                parts = torch.empty(self.P, *w.shape, dtype=w.dtype, device=w.device)
                self._ag(parts, w)
                w = parts.view(-1, w.shape[1])
            out.append(w[:self.sizes[l + 1], :self.sizes[l]].double().cpu())
        return out
