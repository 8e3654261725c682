"""Row-sharded tensor parallelism -- the reference's model-parallel scheme, on RCCL.

The reference splits every layer's neuron rows across MPI ranks / GPU streams, computes
its slice of each layer, and re-assembles the activations, deltas AND the full weight
matrices with all-gathers after every layer and every update (ann.c:912-1860,
cuda_ann.cu:533-2898).  Here, per layer l with rows R_r owned by rank r:

  forward   H_l[:, R_r] = f(H_{l-1} . W_l[R_r]^T)        (gfx950 MFMA GEMM, local)
            H_l = all_gather(H_l[:, R_r])                 (features concatenated)
  output    every rank has the full logits -> identical softmax / loss / delta_L
  backward  P_r = delta_l[:, R_r] . W_l[R_r]              (local MFMA GEMM, FP32)
            delta_{l-1} = all_reduce_sum(P_r) * f'(H_{l-1})
  gradient  G_l[R_r] = delta_l[:, R_r]^T . H_{l-1}        (local, no communication)
  update    on the local rows only

so weights are never all-gathered (the reference moved N_l x M_l weights per layer per
step; this moves B x N_l activations and B x M_l partial deltas).  Intended for layers
too wide for one GPU's memory budget; the headline benchmark uses data parallelism.
"""
import torch
import torch.distributed as dist

from .. import ops
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
        P = self.P
        # every layer's rows padded so each rank holds a multiple of 32
        self.Np = [ops.pad_to(sizes[l + 1], 32 * P) for l in range(self.L)]
        self.Nr = [n // P for n in self.Np]
        self.Kp = [ops.pad_to(sizes[0], 32)] + self.Np[:-1]
        full = reference_init(sizes, seed) if init == "reference" else fast_init(sizes, seed)
        dev = self.device
        self.W32, self.V32, self.Wb, self.Wt = [], [], [], []
        for l in range(self.L):
            w = torch.zeros(self.Np[l], self.Kp[l], dtype=torch.float32)
            w[:sizes[l + 1], :sizes[l]] = full[l].float()
            r0 = self.rank * self.Nr[l]
            wl = w[r0:r0 + self.Nr[l]].contiguous().to(dev)
            self.W32.append(wl)
            self.V32.append(torch.zeros_like(wl) if momentum else None)
            self.Wb.append(torch.empty_like(wl, dtype=torch.bfloat16))
            self.Wt.append(torch.empty(self.Kp[l], self.Nr[l], dtype=torch.bfloat16, device=dev))
            ops.cast_weights(self.W32[l], self.Wb[l], self.Wt[l])
        self.H = [torch.empty(self.Bp, self.Np[l], dtype=torch.bfloat16, device=dev) for l in range(self.L - 1)]
        self.Z = torch.empty(self.Bp, self.Np[-1], dtype=torch.float32, device=dev)
        self.D = [torch.empty(self.Bp, self.Np[l], dtype=torch.bfloat16, device=dev) for l in range(self.L)]
        self.stats = torch.zeros(64, 16, dtype=torch.float32, device=dev)

    def _gather_features(self, local, full):
        """full[:, r*n:(r+1)*n] = local of rank r."""
        if self.P == 1:
            full.copy_(local)
            return full
        B, n = local.shape
        parts = torch.empty(self.P * B, n, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(parts, local.contiguous(), group=self.group)
        full.copy_(parts.view(self.P, B, n).permute(1, 0, 2).reshape(full.shape))
        return full

    def train_step(self, X, labels=None, T=None, n_valid=None, lr=0.01, alpha=0.2):
        n_valid = self.Bp if n_valid is None else n_valid
        L = self.L
        # forward
        for l in range(L):
            A = X if l == 0 else self.H[l - 1]
            last = l == L - 1
            loc = ops.gemm_nt(A, self.Wb[l], ops.EPI_NONE if last else ops.EPI_ACT, out_f32=last)
            self._gather_features(loc, self.Z if last else self.H[l])
        # output (replicated)
        t_hi, t_lo = (1.0, 0.0) if self.type == ops.TYPE_SNN else (1.0, -1.0)
        ops.output_delta(self.Z, self.sizes[-1], self.type, self.D[-1], labels=labels, T=T, t_hi=t_hi, t_lo=t_lo,
                         n_valid=n_valid, loss_acc=self.stats[0, 0:1], correct=self.stats[0, 1:2])
        scale = 1.0 / n_valid
        for l in range(L - 1, -1, -1):
            r0 = self.rank * self.Nr[l]
            Dl = self.D[l][:, r0:r0 + self.Nr[l]]
            Hin = X if l == 0 else self.H[l - 1]
            if l > 0:
                part = ops.gemm_nt(Dl, self.Wt[l], ops.EPI_NONE, out_f32=True)  # [B, Kp[l]] partial
                if self.P > 1:
                    dist.all_reduce(part, group=self.group)
                h = self.H[l - 1].float()
                self.D[l - 1].copy_((part * (-0.5 * (h * h - 1.0))).bfloat16())
            G = ops.gemm_tn(Dl, Hin, splits=1)
            ops.sgd_update(self.W32[l], self.V32[l], G, self.Wb[l], self.Wt[l], lr, alpha, scale, self.momentum)

    def full_weights(self):
        """gather the row shards (FP64 host, unpadded) -- checkpointing / tests."""
        out = []
        for l in range(self.L):
            w = self.W32[l]
            if self.P > 1:
                parts = torch.empty(self.P * w.shape[0], w.shape[1], dtype=w.dtype, device=w.device)
                dist.all_gather_into_tensor(parts, w.contiguous(), group=self.group)
                w = parts
            out.append(w[:self.sizes[l + 1], :self.sizes[l]].double().cpu())
        return out
