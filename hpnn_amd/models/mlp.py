"""Bias-free MLP (libhpnn ANN / SNN / LNN) on the gfx950 kernels.

Math (reference SURVEY 2.4; ann.c / snn.c):
  h_l = f(W_l h_{l-1}),  f(x) = 2/(1+e^-x) - 1   (every hidden layer; ANN output too)
  SNN output  o = e^{z-1} / (TINY + sum e^{z-1}),  delta_L = t - o
  ANN output  o = f(z),                             delta_L = (t - o) f'(o)
  hidden      delta_l = (W_{l+1}^T delta_{l+1}) * f'(h_l),  f'(y) = -0.5 (y^2 - 1)
  update      BP : W += lr * G ;  BPM: dW += lr * G; W += dW; dW *= alpha
  with G = mean over the minibatch of delta_l (x) h_{l-1} (batched mode, see
  csrc/cpu/cpu_batched.cpp for the FP64 oracle of exactly these semantics).

This class is a thin binding over the library's batched plan (csrc/gpu/bplan.h, the same
object train_nn's batched engine runs): the plan picks the step structure, the split-K
factors and the grids, declares the device buffers, and launches every kernel.  Python
allocates those buffers as torch tensors (so W32, G, ... are views the tests and the
data-parallel driver use) and passes the current HIP stream, so steps are captured by
torch.cuda.graph.  On CPU tensors (tests without a GPU) the same configuration runs the
per-layer step in the PyTorch emulation of the kernels (hpnn_amd.ops), whatever the mode.
"""
import ctypes
import ctypes.util
import hashlib
import math
import os

import torch

from .. import ops
from .._lib import native

# the value a uint8 input means (1/255: MNIST pixels normalised to [0, 1])
PIXEL_SCALE = float(torch.tensor(float(os.environ.get("HPNN_PIXEL_SCALE", str(1.0 / 255.0))),
                                 dtype=torch.float32).item())

TYPES = {"ANN": ops.TYPE_ANN, "LNN": ops.TYPE_LNN, "SNN": ops.TYPE_SNN}
_MODES = {"": None, "t": "t", "x": "x", "m": "mid", "w": "w"}
_DT = {0: torch.float32, 1: torch.bfloat16, 2: torch.uint8, 3: torch.int32}


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


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return 0 if t is None else t.data_ptr()


class MLP:
    """Network + device state for batched BF16 MFMA training on one GPU.

    sizes: [n_in, h_1, ..., n_out]; net_type: 'ANN' | 'SNN' | 'LNN'.
    batch: per-step (per-GPU) minibatch (padded by the plan: to 128, 256 on the tile path).
    fused: None / True = the fastest structure the plan finds (True: error if none),
    False = per-layer kernels, or one of "t", "x", "mid", "w" (bplan.h).
    """

    def __init__(self, sizes, net_type="SNN", batch=256, device="cuda", momentum=False, weights=None, seed=10958,
                 init="reference", splits=None, fused=None, mid_grid=512):
        self.sizes = list(sizes)
        self.L = len(sizes) - 1
        self.type = TYPES[net_type] if isinstance(net_type, str) else int(net_type)
        self.type_name = net_type if isinstance(net_type, str) else {v: k for k, v in TYPES.items()}[net_type]
        self.device = torch.device(device)
        self.batch = batch
        self.momentum = momentum
        on_gpu = self.device.type == "cuda"
        req = -1 if fused is None or fused is True else (0 if fused is False else ord({"mid": "m"}.get(fused, fused)))
        try:
            self.plan = native().BPlan(self.sizes, self.type, int(batch), bool(momentum), req, list(splits or []),
                                       int(mid_grid), on_gpu)
        except ValueError as e:
            raise ValueError(f"fused={fused!r}: {e}") from None
        cfg = self.plan.config()
        self.cfg = cfg
        self.Bp, self.Kp, self.Np, self.S = cfg["Bp"], cfg["Kp"], cfg["Np"], cfg["S"]
        self.fused_mode = _MODES[cfg["mode"]]
        if fused is True and self.fused_mode is None:
            raise ValueError(f"no fused path for padded dims {self.Kp[0]}-{self.Np}")
        self.fused = self.fused_mode is not None
        self.n_out = sizes[-1]
        self.mid_groups = cfg["mid_groups"]
        # the plan's buffer table -> torch tensors (views), bound to the plan in table order
        self.buf = {}
        for name, layer, dt, shape, zero in self.plan.buffers():
            mk = torch.zeros if zero else torch.empty
            self.buf[(name, layer)] = mk(tuple(shape), dtype=_DT[dt], device=self.device)
        if on_gpu:
            self.plan.bind([t.data_ptr() for t in self.buf.values()])
        b = self.buf
        self.W32 = [b[("W32", l)] for l in range(self.L)]
        self.V32 = [b.get(("V32", l)) for l in range(self.L)]
        self.Wb = [b[("Wb", l)] for l in range(self.L)]
        self.Wt = [b[("Wt", l)] for l in range(self.L)]
        self.slab = [b[("slab", l)] for l in range(self.L)]
        self.H = [b[("H", l)] for l in range(self.L - 1)]
        self.D = [b[("D", l)] for l in range(self.L)]
        self.Z, self.stats, self.grad_flat = b[("Z", -1)], b[("stats", -1)], b[("gflat", -1)]
        self.G, off = [], 0
        for l in range(self.L):
            n = self.Np[l] * self.Kp[l]
            self.G.append(self.grad_flat[off:off + n].view(self.Np[l], self.Kp[l]))
            off += n
        self.midslab, self.midtmp = b.get(("midslab", -1)), b.get(("midtmp", -1))
        self.W0f = b.get(("W0f", -1))
        if weights is None:
            weights = reference_init(sizes, seed) if init == "reference" else fast_init(sizes, seed)
        for l in range(self.L):
            self.W32[l][:sizes[l + 1], :sizes[l]].copy_(weights[l].to(torch.float32))
        self.refresh_bf16()

    # ------------------------------------------------------------------ helpers
    @property
    def _gpu(self):
        return self.device.type == "cuda"

    @property
    def tn_update(self):
        """the optimizer step in the 8-phase TN gradient's epilogue where it applies (plan)"""
        return self.plan.tn_update

    @tn_update.setter
    def tn_update(self, on):
        self.plan.tn_update = bool(on)

    def _tn_update_ok(self, l):
        return self.plan.tn_update_ok(int(l))

    @staticmethod
    def _pick_splits(N, K, Bp):
        """the plan's split-K rule (bplan.cpp BPlan::pick_splits)"""
        return native().BPlan.pick_splits(N, K, Bp)

    def refresh_bf16(self):
        """BF16 compute copies (and the fragment-major W0) from the FP32 masters"""
        if self._gpu:
            self.plan.cast_weights(_stream())
            return
        for l in range(self.L):
            ops.cast_weights(self.W32[l], self.Wb[l], self.Wt[l], self.W0f if l == 0 else None)

    def host_weights(self):
        """FP64 [N, M] weights (unpadded), for kernel.opt dumps / parity checks."""
        return [self.W32[l][:self.sizes[l + 1], :self.sizes[l]].double().cpu() for l in range(self.L)]

    def prepare_input(self, X, pixel_scale=None):
        """[n, n_in] -> the plan's input layout on the device, >= Bp rows (zero padding).

        X float/double: the values as given (BF16).  X uint8 (8-bit pixel data, e.g. MNIST
        images): the network sees bf16(X * PIXEL_SCALE) (1/255; HPNN_PIXEL_SCALE overrides, 1 =
        the raw 0..255 values the reference's pmnist writes).  Layouts (BPlan.input_layout):
        the tile path ("t") takes the batch fragment-major ([Bp/32, Kp0/16, 64, 8],
        ops.to_fragment_major; 8-bit pixels kept as bytes, exact integers in the MFMAs with
        the scale on the accumulators); "x" takes row-major BF16 plus, for 8-bit data, a
        fragment-major copy of the bytes (attribute `hpnn_fm`) for the first-layer gradient;
        every other mode row-major BF16.  pixel_scale overrides PIXEL_SCALE for this batch
        (1.0: the bytes are the values, as train_nn takes integer 0..255 data)."""
        ps = PIXEL_SCALE if pixel_scale is None else float(pixel_scale)
        Xd = X.to(self.device)
        n = Xd.shape[0]
        layout = self.cfg["input_layout"] if self._gpu else 0
        rows = max(self.Bp, ops.pad_to(n, 256 if layout == 1 else 128))
        u8 = Xd.dtype == torch.uint8
        if layout == 1:
            src = torch.zeros(rows, self.Kp[0], dtype=torch.uint8 if u8 else torch.bfloat16, device=self.device)
            if u8:
                src[:n, :Xd.shape[1]] = Xd
            else:
                ops.pack_bf16(Xd.contiguous(), src)
            out = ops.to_fragment_major(src).view(rows // 32, self.Kp[0] // 16, 64, 8)
            out.hpnn_fm_scale = ps if u8 else 1.0
            return out
        out = torch.empty(rows, self.Kp[0], dtype=torch.bfloat16, device=self.device)
        if u8:
            b = torch.zeros(rows, self.Kp[0], dtype=torch.uint8, device=self.device)
            b[:n, :Xd.shape[1]] = Xd
            out.copy_((b.float() * ps).bfloat16())  # the same rounding as the kernels'
            if layout == 2:
                out.hpnn_fm = ops.to_fragment_major(b)
                out.hpnn_fm_scale = ps
            return out
        ops.pack_bf16(Xd.contiguous(), out)
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
        """the fragment-major copy of a prepared batch X the first-layer gradient streams, or None"""
        if self._is_fm(X):
            return X if X.shape[0] * 32 >= self.Bp else None
        Xg = getattr(X, "hpnn_fm", None)
        if Xg is None or X.shape[0] < self.Bp or Xg.numel() != X.shape[0] * self.Kp[0]:
            return None
        return Xg

    def _x(self, X):
        """(x, xg, u8, scale) plan arguments of a prepared batch; checks it has >= Bp rows"""
        if self._is_fm(X):
            if self.fused_mode != "t" or X.shape[0] * 32 < self.Bp or X.shape[1] * 16 != self.Kp[0]:
                raise ValueError(f"fragment-major batch {tuple(X.shape)} does not fit this plan "
                                 f"(mode {self.fused_mode}, Bp {self.Bp}, Kp0 {self.Kp[0]})")
            u8 = X.dtype == torch.uint8
            return X.data_ptr(), 0, int(u8), float(getattr(X, "hpnn_fm_scale", 1.0))
        if self.fused_mode == "t":
            raise ValueError("the tile path takes fragment-major batches (MLP.prepare_input)")
        if X.shape[0] < self.Bp or X.shape[1] != self.Kp[0] or X.stride(0) != self.Kp[0]:
            raise ValueError(f"batch {tuple(X.shape)} does not fit this plan (Bp {self.Bp}, Kp0 {self.Kp[0]})")
        xg = self._fm_input(X) if self.fused_mode == "x" else None
        # mode x: the u8 flag describes the fragment-major copy (8-bit pixels or BF16)
        return (X.data_ptr(), _p(xg), int(xg is not None and xg.dtype == torch.uint8),
                float(getattr(X, "hpnn_fm_scale", 1.0)))

    @staticmethod
    def _tgt(labels, T):
        return _p(labels), _p(T), (T.stride(0) if T is not None else 0)

    def _t_hilo(self):
        return (1.0, 0.0) if self.type == ops.TYPE_SNN else (1.0, -1.0)

    # ------------------------------------------------------------------ phases
    def forward(self, X):
        X = self._rowmajor(X)
        if self._gpu:
            self.plan.forward(X.data_ptr(), _stream())
            return self.Z
        for l in range(self.L):
            A = X if l == 0 else self.H[l - 1]
            if l == self.L - 1:
                ops.gemm_nt(A, self.Wb[l], ops.EPI_NONE, out_f32=True, out=self.Z)
            else:
                ops.gemm_nt(A, self.Wb[l], ops.EPI_ACT, out=self.H[l])
        return self.Z

    def output(self, labels=None, T=None, n_valid=None):
        n_valid = self.Bp if n_valid is None else int(n_valid)
        if self._gpu:
            self.plan.output(*self._tgt(labels, T), n_valid, 0, 0, True, _stream())
            return
        t_hi, t_lo = self._t_hilo()
        ops.output_delta(self.Z, self.n_out, self.type, self.D[-1], labels=labels, T=T, t_hi=t_hi, t_lo=t_lo,
                         n_valid=n_valid, loss_acc=self.stats[0, 0:1], correct=self.stats[0, 1:2])

    def backward_layer(self, l):
        """D[l-1] = (D[l] @ W_l) * f'(H[l-1]) (uses pre-update W_l^T)."""
        if self._gpu:
            self.plan.backward_layer(l, _stream())
            return
        ops.gemm_nt(self.D[l], self.Wt[l], ops.EPI_DACT, aux=self.H[l - 1], out=self.D[l - 1])

    def grad_layer(self, l, X, reduce=False):
        if self._gpu:
            self.plan.grad_layer(l, *self._x(X), bool(reduce), _stream())
            return
        Hin = X if l == 0 else self.H[l - 1]
        if reduce and self.S[l] == 1:
            ops.gemm_tn(self.D[l], Hin, splits=1, out=self.G[l].unsqueeze(0))
            return
        ops.gemm_tn(self.D[l], Hin, splits=self.S[l], out=self.slab[l])
        if reduce:
            ops.reduce_slabs(self.slab[l], self.G[l])

    def update_layer(self, l, lr, alpha, scale, from_G=False):
        if self._gpu:
            self.plan.update_layer(l, float(lr), float(alpha), float(scale), bool(from_G), _stream())
            return
        G = self.G[l] if from_G else self.slab[l]
        ops.sgd_update(self.W32[l], self.V32[l], G, self.Wb[l], self.Wt[l], lr, alpha, scale, self.momentum)

    def update_all(self, lr, alpha, scale, grads=None):
        """every layer's optimizer step from the flat gradient buffer (the data-parallel
        all-reduce result), one launch"""
        if self._gpu:
            self.plan.update_flat(self.grad_flat.data_ptr(), float(lr), float(alpha), float(scale), _stream())
            return
        for l in range(self.L):
            self.update_layer(l, lr, alpha, scale, from_G=True)

    def front(self, X, labels=None, T=None, n_valid=None):
        """fused modes: X -> the deltas (+ the [G1 | G2] block slabs), one launch"""
        n_valid = self.Bp if n_valid is None else int(n_valid)
        if not (self._gpu and self.fused):
            raise RuntimeError("front() needs a fused plan on a GPU")
        self.plan.front(*self._x(X), *self._tgt(labels, T), n_valid, _stream())

    _fused_front = front

    def backward_grads(self, X, labels=None, T=None, n_valid=None, reduce=True, on_ready=None):
        """forward + backward of one minibatch, the weight gradients summed into self.G[l]
        (the all-reduce buckets); on_ready(l) is called as soon as layer l's gradient is final
        (layers become ready from the last to the first)."""
        n_valid = self.Bp if n_valid is None else int(n_valid)
        if self._gpu:
            def ready(lo, hi):
                if on_ready:
                    for l in range(hi, lo - 1, -1):
                        on_ready(l)
                return True
            self.plan.grads(*self._x(X), *self._tgt(labels, T), n_valid, ready, _stream())
            return
        self.forward(X)
        self.output(labels=labels, T=T, n_valid=n_valid)
        for l in range(self.L - 1, -1, -1):
            if l > 0:
                self.backward_layer(l)
            self.grad_layer(l, X, reduce=True)
            if on_ready:
                on_ready(l)

    def grads_slabs(self, X, labels=None, T=None, n_valid=None, dst=None):
        """fused modes: front + first-layer gradient with the gradient left unreduced; returns
        [(address, slab stride, slabs, floats)] segments for the xGMI all-reduce's copy-in.
        dst = (address, selector address, half stride in floats) -- the all-reduce's own
        buffer (NativeComm.xar_local): when G0 reduces in-kernel the gradient goes there and
        the result is [] (nothing to copy in)"""
        n_valid = self.Bp if n_valid is None else int(n_valid)
        d, sel, alt = dst if dst is not None else (0, 0, 0)
        return self.plan.grads_slabs(*self._x(X), *self._tgt(labels, T), n_valid, _stream(), d, sel, alt)

    def train_step(self, X, labels=None, T=None, n_valid=None, lr=0.01, alpha=0.2):
        """One minibatch fwd + bwd + update on the current stream (no host sync)."""
        n_valid = self.Bp if n_valid is None else int(n_valid)
        if self._gpu:
            self.plan.step(*self._x(X), *self._tgt(labels, T), n_valid, float(lr), float(alpha), _stream())
            return
        scale = 1.0 / n_valid
        self.forward(X)
        self.output(labels=labels, T=T, n_valid=n_valid)
        for l in range(self.L - 1, -1, -1):
            if l > 0:
                self.backward_layer(l)  # pre-update W_l^T, before layer l's step below
            self.grad_layer(l, X)
            self.update_layer(l, lr, alpha, scale)

    def predict(self, X, n_valid=None):
        """network outputs [n_valid, n_out] (fp32)."""
        n_valid = (X.shape[0] * 32 if self._is_fm(X) else X.shape[0]) if n_valid is None else n_valid
        n_valid = min(int(n_valid), self.Bp)
        O = torch.empty(self.Bp, self.Np[-1], dtype=torch.float32, device=self.device)
        if self._gpu:
            self.plan.predict(self._rowmajor(X).data_ptr(), n_valid, O.data_ptr(), O.stride(0), _stream())
            return O[:n_valid, :self.n_out]
        self.forward(X)
        Tz = torch.zeros(self.Bp, self.n_out, dtype=torch.float32, device=self.device)
        ops.output_delta(self.Z, self.n_out, self.type, self.D[-1], T=Tz, n_valid=n_valid, O=O)
        return O[:n_valid, :self.n_out]

    def healthy(self):
        """False when an in-kernel hand-off (the fused G0's split-K tickets, a fused TN
        gradient's tickets, the wide front's tile pair) timed out since the model was made:
        that step used partial sums (synchronises the current stream)."""
        if not self._gpu:
            return True
        return self.plan.health(_stream()) == 0

    def weights_digest(self, which=3):
        """64-bit digest of the weights (1: BF16 copies, 2: FP32 masters, 3: both); data-
        parallel replicas hold bitwise-identical weights, so equal digests (synchronises)."""
        if self._gpu:
            return int(self.plan.weights_digest(int(which), _stream()))
        # a keyless, process-independent hash (Python's hash() of bytes is salted per process,
        # so replicas in different processes would never agree)
        h = hashlib.blake2b(digest_size=8)
        for l in range(self.L):
            ts = ([self.Wb[l], self.Wt[l]] if which & 1 else []) + ([self.W32[l]] if which & 2 else [])
            for t in ts:
                h.update(t.contiguous().view(-1).view(torch.int16 if t.element_size() == 2
                                                      else torch.int32).cpu().numpy().tobytes())
        return int.from_bytes(h.digest(), "little")

    def reset_stats(self):
        self.stats.zero_()

    def read_stats(self):
        s = self.stats.cpu()
        return float(s[:, 0].double().sum()), int(s[:, 1].contiguous().view(torch.int32).long().sum())
