"""Bias-free MLP (libhpnn ANN / SNN / LNN) on the gfx950 kernels.

Math (reference SURVEY 2.4; ann.c / snn.c):
  h_l = f(W_l h_{l-1}),  f(x) = 2/(1+e^-x) - 1   (every hidden layer; ANN output too)
  SNN output  o = e^{z-1} / (TINY + sum e^{z-1}),  delta_L = t - o
  ANN output  o = f(z),                             delta_L = (t - o) f'(o)
  hidden      delta_l = (W_{l+1}^T delta_{l+1}) * f'(h_l),  f'(y) = -0.5 (y^2 - 1)
  update      BP : W += lr * G ;  BPM: dW += lr * G; W += dW; dW *= alpha
  with G = mean over the minibatch of delta_l (x) h_{l-1} (batched mode, see
  csrc/cpu/cpu_batched.cpp for the FP64 oracle of exactly these semantics).

Device layout (csrc/gpu/kernels.h): activations [batch, features] BF16, feature dims
padded to 32, batch padded to 128; W [N, K] BF16 + W^T [K, N] BF16 for the dX GEMM;
FP32 master weights and momentum; FP32 split-K gradient slabs.
"""
import ctypes
import ctypes.util
import math
import os

import torch

from .. import ops

# uint8 (pixel) input on the fused path: fragment-major 8-bit copy for the G0 kernel
# (HPNN_G0_FM_U8=0 disables: LDS-staged TN GEMM on the BF16 batch)
_G0_FM_U8 = os.environ.get("HPNN_G0_FM_U8", "1") == "1"
# the value a uint8 input means (1/255: MNIST pixels normalised to [0, 1])
PIXEL_SCALE = float(torch.tensor(float(os.environ.get("HPNN_PIXEL_SCALE", str(1.0 / 255.0))),
                                 dtype=torch.float32).item())
# HPNN_TILE=0: the 32-sample pipelined front (mlp3_fused, "x") instead of the 256-sample
# tile kernel (mlp3_tile, "t") on eligible MNIST-shaped nets
_TILE = os.environ.get("HPNN_TILE", "1") != "0"
# HPNN_WIDE=0: the per-layer kernels instead of the wide-input front ("w") for
# 4096 -> 256 -> 256 (padded) nets
_WIDE = os.environ.get("HPNN_WIDE", "1") != "0"

TYPES = {"ANN": ops.TYPE_ANN, "LNN": ops.TYPE_LNN, "SNN": ops.TYPE_SNN}


def reference_init(sizes, seed):
    """Bit-identical to libhpnn ann_generate (ann.c:632-766): glibc srandom(seed),
    w = 2 (random()/RAND_MAX - 0.5) / sqrt(M), hidden layers first, row-major."""
    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    libc.random.restype = ctypes.c_long
    libc.srandom(ctypes.c_uint(seed))
    rand_max = 2147483647.0
    out = []
    for l in range(len(sizes) - 1):
        M, N = sizes[l], sizes[l + 1]
        n = N * M
        if n > 4_000_000:
            raise ValueError("reference_init is meant for small nets; use init='fast'")
        w = torch.tensor([libc.random() for _ in range(n)], dtype=torch.float64)
        w = 2.0 * (w / rand_max - 0.5) / math.sqrt(M)
        out.append(w.view(N, M))
    return out


def fast_init(sizes, seed):
    """Same distribution U(-1,1)/sqrt(M) from torch's generator (large benchmark nets)."""
    g = torch.Generator().manual_seed(seed)
    return [((torch.rand(sizes[l + 1], sizes[l], generator=g, dtype=torch.float64) - 0.5) * 2.0
             / math.sqrt(sizes[l])) for l in range(len(sizes) - 1)]


class MLP:
    """Network + device state for batched BF16 MFMA training on one GPU.

    sizes: [n_in, h_1, ..., n_out]; net_type: 'ANN' | 'SNN' | 'LNN'.
    batch: per-step (per-GPU) minibatch; padded to a multiple of 128 internally.
    """

    def __init__(self, sizes, net_type="SNN", batch=256, device="cuda", momentum=False, weights=None, seed=10958,
                 init="reference", splits=None, fused=None, mid_grid=512):
        self.sizes = list(sizes)
        self.L = len(sizes) - 1
        self.type = TYPES[net_type] if isinstance(net_type, str) else int(net_type)
        self.type_name = net_type if isinstance(net_type, str) else {v: k for k, v in TYPES.items()}[net_type]
        self.device = torch.device(device)
        self.batch = batch
        self.Bp = ops.pad_to(batch, 128)
        self.momentum = momentum
        self.tn_update = os.environ.get("HPNN_TN_UPD", "1") != "0"
        self.Kp = [ops.pad_to(sizes[l], 32) for l in range(self.L)]
        self.Np = [ops.pad_to(sizes[l + 1], 32) for l in range(self.L)]
        self.n_out = sizes[-1]
        if weights is None:
            weights = reference_init(sizes, seed) if init == "reference" else fast_init(sizes, seed)
        dev = self.device
        self.W32, self.V32, self.Wb, self.Wt, self.slab, self.S = [], [], [], [], [], []
        for l in range(self.L):
            N, K = self.Np[l], self.Kp[l]
            w = torch.zeros(N, K, dtype=torch.float32)
            w[:sizes[l + 1], :sizes[l]] = weights[l].to(torch.float32)
            self.W32.append(w.to(dev))
            self.V32.append(torch.zeros(N, K, dtype=torch.float32, device=dev) if momentum else None)
            self.Wb.append(torch.empty(N, K, dtype=torch.bfloat16, device=dev))
            self.Wt.append(torch.empty(K, N, dtype=torch.bfloat16, device=dev))
            S = splits[l] if splits else self._pick_splits(N, K, self.Bp)
            self.S.append(S)
            self.slab.append(torch.empty(S, N, K, dtype=torch.float32, device=dev))
        # flat FP32 gradient buffer (one view per layer: the DP all-reduce buckets)
        sizes_g = [self.Np[l] * self.Kp[l] for l in range(self.L)]
        self.grad_flat = torch.zeros(sum(sizes_g), dtype=torch.float32, device=dev)
        self.G, off = [], 0
        for l in range(self.L):
            self.G.append(self.grad_flat[off:off + sizes_g[l]].view(self.Np[l], self.Kp[l]))
            off += sizes_g[l]
        self.H = [torch.empty(self.Bp, self.Np[l], dtype=torch.bfloat16, device=dev) for l in range(self.L - 1)]
        self.D = [torch.empty(self.Bp, self.Np[l], dtype=torch.bfloat16, device=dev) for l in range(self.L)]
        self.Z = torch.empty(self.Bp, self.Np[-1], dtype=torch.float32, device=dev)
        # loss / accuracy: 64 slots x 16 floats ([0] loss sum, [1] hits as uint32 bits),
        # see HPNN_STAT_SLOTS in csrc/gpu/kernels.h
        self.stats = torch.zeros(64, 16, dtype=torch.float32, device=dev)
        # fused 3-layer paths (csrc/gpu/kernels_mlp3.hip) for n_in-128-64-(<=32) nets:
        #   "x"   : mlp3_fused (X -> delta1 in one kernel, W0 register-resident)
        #   "mid" : gemm_nt layer 0 + mlp3_mid (H1 -> delta1)
        eligible = self.L == 3 and tuple(self.Np) == ops.MLP3_DIMS
        x_ok = eligible and self.Kp[0] in ops.MLP3F_K0
        t_ok = eligible and self.Kp[0] in ops.MLP3T_K0 and self.Bp % ops.MLP3T_TILE == 0
        #   "w"   : wide2_front (K0 = 4096 -> 256 -> 256: X -> H0, delta2, delta1 in one kernel)
        w_ok = (self.L == 2 and tuple(self.Np) == (256, 256) and self.Kp[0] in ops.WIDE2_K0
                and self.Bp % ops.WIDE2_TILE == 0)
        if fused is None or fused is True:
            mode = "t" if (t_ok and _TILE) else ("x" if x_ok else ("mid" if eligible else None))
            if mode is None and w_ok and _WIDE:
                mode = "w"
            if fused is True and mode is None:
                raise ValueError(f"fused path needs padded dims {ops.MLP3_DIMS}, got {self.Np}")
        elif fused in ("x", "mid", "t", "w"):
            if not {"x": x_ok, "mid": eligible, "t": t_ok, "w": w_ok}[fused]:
                raise ValueError(f"fused={fused!r} not available for dims {self.Kp[0]}-{self.Np}")
            mode = fused
        else:
            mode = None
        self.fused_mode = mode
        self.fused = mode is not None
        self.W0f = None
        self.wide_ws = ops.Wide2Workspace(self.Bp, self.Kp[0], dev) if mode == "w" else None
        if mode == "mid":
            grid = max(1, min(mid_grid, self.Bp // 64))
            self.midslab = torch.empty(grid, ops.MLP3_SLAB, dtype=torch.float32, device=dev)
            self.midtmp = torch.empty(16 * self.midslab.shape[1], dtype=torch.float32, device=dev)
        elif mode in ("x", "t"):
            grid = ops.mlp3_fused_grid(self.Bp, dev) if mode == "x" else ops.mlp3_tile_grid(self.Bp, dev)
            self.midslab = torch.empty(grid, ops.MLP3_SLAB, dtype=torch.float32, device=dev)
            self.mid_groups = min(16, grid)
            self.midtmp = torch.empty(16 * ops.MLP3_SLAB, dtype=torch.float32, device=dev)
            self.W0f = torch.empty(self.Np[0] * self.Kp[0], dtype=torch.bfloat16, device=dev)
        self.refresh_bf16()

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _pick_splits(N, K, Bp):
        """split-K factor of the weight-gradient GEMM (mirrors csrc/gpu/gpu_engine.cpp
        pick_splits): about one workgroup per CU (256 on MI355X; measured 76.1 us/step
        at 48 splits vs 79.7 us at 64 and 78.9 us at 96 for MNIST) so that every CU
        streams the same share -- the kernel accepts uneven splits --, at least 512 batch
        rows per split, and a multiple of 8 for the XCD-aware block order.
        HPNN_TN_SPLITS forces a value (tuning)."""
        tn = 128 if N % 128 == 0 else (64 if N % 64 == 0 else 32)
        tm = next(t for t in (128, 160, 96, 64, 32) if K % t == 0)
        tiles = (N // tn) * (K // tm)
        forced = int(os.environ.get("HPNN_TN_SPLITS", "0"))
        if forced > 0:
            return max(1, min(forced, Bp // 64)) if Bp % 64 == 0 else 1
        s8 = MLP._splits_8ph(N, K, Bp)
        if s8:
            return s8
        rows = int(os.environ.get("HPNN_TN_ROWS", "512"))
        s = (256 + tiles // 2) // max(tiles, 1)
        s = min(s, Bp // rows)
        if s >= 8:
            s -= s % 8
        return max(1, s)

    @staticmethod
    def _splits_8ph(N, K, Bp):
        """split count that puts a weight gradient with 256x256 tiles on the 8-phase TN kernel
        (kernels_8ph.hip: >= 256 workgroups, an even number of 64-row units per split), or 0.
        RRUFF-shaped 4096 -> 256 first layer over 16384 rows: 16 splits, 162-164 us/step vs
        171-173 with 4 splits on the 128x128 kernel (scripts/gpu_rruff_splits.sh)."""
        if N % 256 or K % 256 or Bp % 128 or os.environ.get("HPNN_TN_8PH", "1") == "0":
            return 0
        t8, units = (N // 256) * (K // 256), Bp // 64
        for s in range(max(1, -(-256 // t8)), 2 * max(1, -(-256 // t8)) + 1):
            if units % s == 0 and (units // s) % 2 == 0:
                return s
        return 0

    def refresh_bf16(self):
        for l in range(self.L):
            ops.cast_weights(self.W32[l], self.Wb[l], self.Wt[l], self.W0f if l == 0 else None)

    def host_weights(self):
        """FP64 [N, M] weights (unpadded), for kernel.opt dumps / parity checks."""
        return [self.W32[l][:self.sizes[l + 1], :self.sizes[l]].double().cpu() for l in range(self.L)]

    def prepare_input(self, X):
        """[n, n_in] -> padded BF16 [Bp, Kp0] device tensor.

        X float/double: the values as given.  X uint8 (8-bit pixel data, e.g. MNIST images):
        the network sees bf16(X * PIXEL_SCALE) (PIXEL_SCALE = 1/255, the usual [0, 1]
        normalisation; HPNN_PIXEL_SCALE overrides, 1 = raw 0..255 values as the reference's
        pmnist writes them), and on the fused MNIST-shape path ("x") the returned tensor
        also carries the pixels themselves in fragment-major order (attribute `hpnn_fm`,
        ops.to_fragment_major, one byte per value): the first-layer gradient kernel
        (csrc/gpu/kernels_g0.hip) streams that copy -- half the bytes of the BF16 batch, no
        LDS transposes -- and converts it exactly as above.  (The tile path, "t", takes the
        batch itself fragment-major: _prepare_fm.)"""
        Xd = X.to(self.device)
        if self.fused_mode == "t":
            return self._prepare_fm(Xd)
        rows = ops.pad_to(X.shape[0], 128)
        out = torch.empty(rows, self.Kp[0], dtype=torch.bfloat16, device=self.device)
        if Xd.dtype == torch.uint8:
            u8 = torch.zeros(rows, self.Kp[0], dtype=torch.uint8, device=self.device)
            u8[:X.shape[0], :X.shape[1]] = Xd
            out.copy_((u8.float() * PIXEL_SCALE).bfloat16())  # the same rounding as the kernel's
            if self.fused_mode == "x" and _G0_FM_U8:
                out.hpnn_fm = ops.to_fragment_major(u8)
                out.hpnn_fm_scale = PIXEL_SCALE
            return out
        ops.pack_bf16(Xd.contiguous(), out)
        return out

    def _prepare_fm(self, Xd):
        """tile path ("t"): the batch itself fragment-major ([rows/32, Kp0/16, 64, 8],
        ops.to_fragment_major), 8-bit pixels kept as bytes (the kernels use bf16(x *
        PIXEL_SCALE)), anything else as BF16.  Both the front kernel and the first-layer
        gradient kernel stream this one buffer."""
        rows = ops.pad_to(Xd.shape[0], ops.MLP3T_TILE)
        if Xd.dtype == torch.uint8:
            u8 = torch.zeros(rows, self.Kp[0], dtype=torch.uint8, device=self.device)
            u8[:Xd.shape[0], :Xd.shape[1]] = Xd
            out = ops.to_fragment_major(u8).view(rows // 32, self.Kp[0] // 16, 64, 8)
            out.hpnn_fm_scale = PIXEL_SCALE
        else:
            b = torch.empty(rows, self.Kp[0], dtype=torch.bfloat16, device=self.device)
            ops.pack_bf16(Xd.contiguous(), b)
            out = ops.to_fragment_major(b).view(rows // 32, self.Kp[0] // 16, 64, 8)
            out.hpnn_fm_scale = 1.0
        out.hpnn_fm_rows = rows
        return out

    @staticmethod
    def _is_fm(X):
        return X.dim() >= 4

    def _rowmajor(self, X):
        """row-major BF16 [rows, Kp0] view of a prepared batch (fragment-major input of the
        tile path is converted; the per-layer kernels need rows)"""
        if not self._is_fm(X):
            return X
        rows = X.shape[0] * 32
        R = ops.from_fragment_major(X, rows, X.shape[1] * 16)
        if X.dtype == torch.uint8:
            return (R.float() * getattr(X, "hpnn_fm_scale", PIXEL_SCALE)).bfloat16()
        return R.contiguous()

    def _fm_input(self, X):
        """the fragment-major copy of a prepared batch X (prepare_input), or None"""
        if self._is_fm(X):
            return X if X.shape[0] * 32 == self.Bp else None
        Xg = getattr(X, "hpnn_fm", None)
        if Xg is None or X.shape[0] != self.Bp or Xg.numel() != X.shape[0] * self.Kp[0]:
            return None
        return Xg

    # ------------------------------------------------------------------ phases
    def forward(self, X):
        X = self._rowmajor(X)
        for l in range(self.L):
            A = X if l == 0 else self.H[l - 1]
            if l == self.L - 1:
                ops.gemm_nt(A, self.Wb[l], ops.EPI_NONE, out_f32=True, out=self.Z)
            else:
                ops.gemm_nt(A, self.Wb[l], ops.EPI_ACT, out=self.H[l])
        return self.Z

    def output(self, labels=None, T=None, n_valid=None, O=None):
        t_hi, t_lo = (1.0, 0.0) if self.type == ops.TYPE_SNN else (1.0, -1.0)
        ops.output_delta(self.Z, self.n_out, self.type, self.D[-1], labels=labels, T=T, t_hi=t_hi, t_lo=t_lo,
                         n_valid=n_valid, O=O, loss_acc=self.stats[0, 0:1], correct=self.stats[0, 1:2])

    def backward_layer(self, l):
        """D[l-1] = (D[l] @ W_l) * f'(H[l-1]) (uses pre-update W_l^T)."""
        ops.gemm_nt(self.D[l], self.Wt[l], ops.EPI_DACT, aux=self.H[l - 1], out=self.D[l - 1])

    def grad_layer(self, l, X, reduce=False):
        Hin = X if l == 0 else self.H[l - 1]
        Xg = self._fm_input(X) if l == 0 and self.fused_mode in ("x", "t") else None
        if Xg is not None:  # delta1 came fragment-major from the fused front
            ops.gemm_fm_direct(self.D[0], Xg, self.Np[0], self.Kp[0], splits=self.S[0], out=self.slab[0],
                               hscale=getattr(X, "hpnn_fm_scale", 1.0))
        elif reduce and self.S[l] == 1:
            # one split: the GEMM writes the all-reduce bucket itself (no slab copy)
            ops.gemm_tn(self.D[l], Hin, splits=1, out=self.G[l].unsqueeze(0))
            return
        else:
            ops.gemm_tn(self.D[l], Hin, splits=self.S[l], out=self.slab[l])
        if reduce:
            ops.reduce_slabs(self.slab[l], self.G[l])

    def update_layer(self, l, lr, alpha, scale, from_G=False):
        G = self.G[l] if from_G else self.slab[l]
        if l == 0 and self.W0f is not None:
            ops.sgd_update_multi([(self.W32[0], self.V32[0], G, self.Wb[0], self.Wt[0], self.W0f)], lr, alpha,
                                 scale, self.momentum)
            return
        ops.sgd_update(self.W32[l], self.V32[l], G, self.Wb[l], self.Wt[l], lr, alpha, scale, self.momentum)

    def update_all(self, lr, alpha, scale, grads):
        """every layer's optimizer step in one launch; grads[l]: [S, N, K] (view) or [N, K]"""
        ops.sgd_update_multi([(self.W32[l], self.V32[l], grads[l], self.Wb[l], self.Wt[l],
                               self.W0f if l == 0 else None) for l in range(self.L)], lr, alpha, scale, self.momentum)

    def _mid_group_views(self):
        """[G1 | G2] partial sums in midtmp as [groups, N, K] views for update_all"""
        g = self.mid_groups
        t = self.midtmp[:g * ops.MLP3_SLAB].view(g, ops.MLP3_SLAB)
        n1 = self.Np[1] * self.Kp[1]
        return (t[:, :n1].view(g, self.Np[1], self.Kp[1]),
                t[:, n1:n1 + self.Np[2] * self.Kp[2]].view(g, self.Np[2], self.Kp[2]))

    def _t_hilo(self):
        return (1.0, 0.0) if self.type == ops.TYPE_SNN else (1.0, -1.0)

    def backward_grads(self, X, labels=None, T=None, n_valid=None, reduce=False, on_ready=None):
        """forward + backward of one minibatch.  Weight gradients end in self.slab[l]
        (split-K slabs) or, with reduce=True, summed in self.G[l] (the all-reduce
        buckets).  on_ready(l) is called as soon as layer l's gradient is final (layers
        become ready from the last to the first)."""
        n_valid = self.Bp if n_valid is None else n_valid
        if self.fused_mode == "w":
            self._fused_front(X, labels, T, n_valid)
            for l in (1, 0):
                self.grad_layer(l, X, reduce=reduce)
                if on_ready:
                    on_ready(l)
            return
        if self.fused:
            self._fused_front(X, labels, T, n_valid)
            # G1 | G2 are contiguous in grad_flat, exactly the per-block slab layout
            g12 = self.grad_flat[self.G[1].data_ptr() // 4 - self.grad_flat.data_ptr() // 4:]
            ops.reduce_slabs2(self.midslab, g12[:self.midslab.shape[1]], self.midtmp)
            if on_ready:
                on_ready(2)
                on_ready(1)
            self.grad_layer(0, X, reduce=reduce)
            if on_ready:
                on_ready(0)
            return
        self.forward(X)
        self.output(labels=labels, T=T, n_valid=n_valid)
        for l in range(self.L - 1, -1, -1):
            if l > 0:
                self.backward_layer(l)
            self.grad_layer(l, X, reduce=reduce)
            if on_ready:
                on_ready(l)

    def _fused_front(self, X, labels, T, n_valid):
        """X -> delta1 (self.D[0]) + per-block [G1 | G2] slabs (self.midslab)"""
        t_hi, t_lo = self._t_hilo()
        kw = dict(labels=labels, T=T, t_hi=t_hi, t_lo=t_lo, n_valid=n_valid, loss_acc=self.stats[0, 0:1],
                  correct=self.stats[0, 1:2])
        if self.fused_mode == "w":
            ops.wide2_front(X, self.Wb[0], self.Wb[1], self.Wt[1], self.H[0], self.D[1], self.D[0], self.wide_ws,
                            self.n_out, self.type, **kw)
        elif self.fused_mode == "t":
            ops.mlp3_tile(X, self.Kp[0], self.Wb[0], self.W0f, self.Wb[1], self.Wb[2], self.Wt[2], self.D[0],
                          self.midslab, self.n_out, self.type, xscale=getattr(X, "hpnn_fm_scale", 1.0), **kw)
        elif self.fused_mode == "x":
            ops.mlp3_fused(X, self.Wb[0], self.W0f, self.Wb[1], self.Wb[2], self.D[0], self.midslab, self.n_out,
                           self.type, d1_fm=self._fm_input(X) is not None, **kw)
        else:
            ops.gemm_nt(X, self.Wb[0], ops.EPI_ACT, out=self.H[0])
            ops.mlp3_mid(self.H[0], self.Wb[1], self.Wt[1], self.Wb[2], self.Wt[2], self.D[0], self.midslab,
                         self.n_out, self.type, **kw)

    def _g0_reduce(self, X, groups):
        """first-layer gradient slabs (self.slab[0]) + the first [G1|G2] reduction pass
        (into groups) in one launch, after _fused_front on the same X"""
        Xg = self._fm_input(X)
        if Xg is not None:
            ops.gemm_fm_direct_reduce(self.D[0], Xg, self.Np[0], self.Kp[0], self.S[0], self.slab[0], self.midslab,
                                      self.mid_groups, groups, hscale=getattr(X, "hpnn_fm_scale", 1.0))
        else:
            ops.gemm_tn_reduce(self.D[0], X, self.S[0], self.slab[0], self.midslab, self.mid_groups, groups)

    def train_step(self, X, labels=None, T=None, n_valid=None, lr=0.01, alpha=0.2):
        """One minibatch fwd + bwd + update on the current stream (no host sync)."""
        n_valid = self.Bp if n_valid is None else n_valid
        scale = 1.0 / n_valid
        if self.fused_mode in ("x", "t"):
            # 3 launches: fused front; the G0 GEMM with the first [G1|G2] reduction pass on
            # tail workgroups appended to its grid (they fill the CUs the GEMM tiles leave
            # idle); every layer's update
            self._fused_front(X, labels, T, n_valid)
            groups = self.midtmp[:self.mid_groups * ops.MLP3_SLAB].view(self.mid_groups, ops.MLP3_SLAB)
            self._g0_reduce(X, groups)
            g1, g2 = self._mid_group_views()
            self.update_all(lr, alpha, scale, [self.slab[0], g1, g2])
            return
        if self.fused_mode == "w":
            # one launch up to the deltas, then the per-layer weight gradients and steps (one
            # multi-layer update launch measured no faster: 22.1 us vs 2 x 10.7)
            self._fused_front(X, labels, T, n_valid)
            self._grads_and_steps(X, lr, alpha, scale)
            return
        if self.fused:
            self.backward_grads(X, labels=labels, T=T, n_valid=n_valid)
            self.update_layer(0, lr, alpha, scale)
            self.update_layer(1, lr, alpha, scale, from_G=True)
            self.update_layer(2, lr, alpha, scale, from_G=True)
            return
        self.forward(X)
        self.output(labels=labels, T=T, n_valid=n_valid)
        self._grads_and_steps(X, lr, alpha, scale, backprop=True)

    def _grads_and_steps(self, X, lr, alpha, scale, backprop=False):
        """from the last layer to the first: (backprop: the delta of the layer below, with the
        pre-update W_l^T), the weight gradient and the optimizer step"""
        for l in range(self.L - 1, -1, -1):
            if backprop and l > 0:
                self.backward_layer(l)  # pre-update W_l^T, before layer l's step below
            Hin = X if l == 0 else self.H[l - 1]
            if self._tn_update_ok(l) and ops.gemm_tn_update(self.D[l], Hin, self.W32[l], self.V32[l], self.Wb[l],
                                                             self.Wt[l], lr, alpha, scale, self.momentum):
                continue  # gradient + step in one launch, no gradient in memory
            self.grad_layer(l, X)
            self.update_layer(l, lr, alpha, scale)

    def _tn_update_ok(self, l):
        """layer l's weight gradient and optimizer step can run as one 8-phase TN launch
        (ops.gemm_tn_update): one split, 256x256 tiles, no fragment-major W0 copy to keep;
        tn_update=False (or HPNN_TN_UPD=0) keeps the separate gradient + update kernels.
        Synthetic 8x4096 ANN: see profiles/r2/s5_8ph_gemm.md."""
        return (self.tn_update and self.device.type == "cuda" and self.S[l] == 1 and self.Np[l] % 256 == 0
                and self.Kp[l] % 256 == 0 and self.Bp % 128 == 0 and not (l == 0 and self.W0f is not None))

    def predict(self, X, n_valid=None):
        """network outputs [n_valid, n_out] (fp32)."""
        n_valid = (X.shape[0] * 32 if self._is_fm(X) else X.shape[0]) if n_valid is None else n_valid
        self.forward(X)
        O = torch.empty(self.Bp, self.Np[-1], dtype=torch.float32, device=self.device)
        Tz = torch.zeros(self.Bp, self.n_out, dtype=torch.float32, device=self.device)
        ops.output_delta(self.Z, self.n_out, self.type, self.D[-1], T=Tz, n_valid=n_valid, O=O)
        return O[:n_valid, :self.n_out]

    def reset_stats(self):
        self.stats.zero_()

    def read_stats(self):
        s = self.stats.cpu()
        return float(s[:, 0].double().sum()), int(s[:, 1].contiguous().view(torch.int32).long().sum())
