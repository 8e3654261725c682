"""Data parallelism: one process per GPU, gradient all-reduce over RCCL (xGMI).

Replaces the reference's MPI tier (which replicated the *same* sample on every rank and
all-gathered whole weight matrices after every update) with true data
parallelism: each rank trains on its own minibatch shard, and the FP32 weight gradients
are summed with all-reduce.

Overlap: the backward runs layer L-1 -> 0.  As soon as layer l's weight gradient is
reduced from its split-K slabs into its bucket (a view of one flat FP32 buffer), an
async all-reduce of that bucket is issued; ProcessGroupNCCL runs it on its own stream
that waits only for the work enqueued so far, so it overlaps the backward GEMMs of the
lower layers.  The optimizer kernels then wait (stream-side, no host sync) for their
bucket.  Small consecutive layers are merged into one bucket (`bucket_bytes`) because a
37 KB all-reduce is latency-bound on xGMI.
"""
import os
import sys

import torch
import torch.distributed as dist

from .. import ops

# HPNN_XAR_UPD=0: separate optimizer launch after the xGMI all-reduce (fused MNIST path)
_XAR_UPD = os.environ.get("HPNN_XAR_UPD", "1") == "1"
# HPNN_XAR_LOCAL=0: the G0 launch writes gflat and the all-reduce copies it in (A/B)
_XAR_LOCAL = os.environ.get("HPNN_XAR_LOCAL", "1") == "1"
# HPNN_XAR_G0=0: no exchange inside the first-layer gradient launch (separate all-reduce launch)
_XAR_G0 = os.environ.get("HPNN_XAR_G0", "1") == "1"


class DataParallel:
    """comm: "auto" (libhpnn's native RCCL communicator when the model is on a GPU and the
    group runs on the nccl backend, else torch.distributed), "native", "torch", or "xar"
    (xGMI all-reduce only, no RCCL: several ranks on one GPU in tests).

    grad_comm: "auto" (default): "bf16rs" with more than one rank when the model takes the
    per-layer path and its FP32 gradients exceed 4 MB (the exchange is bandwidth-bound there:
    half the bytes, and each rank steps 1/world of the rows), else "fp32".
    "fp32": the FP32 gradient buckets are all-reduced, every rank
    applies the whole update.  "bf16rs": for layers whose rows split evenly over the ranks,
    the gradient is reduce-scattered in BF16, each rank steps ITS rows of the FP32 master
    weights / momentum (a sharded optimizer), and the BF16 weight rows are all-gathered:
    (W-1)/W x P x (2 + 2) bytes per rank and step instead of the ring all-reduce's
    2 (W-1)/W x P x 4 -- half (the 8 x 4096 synthetic config: 470 vs 940 MB).  The FP32
    masters then live sharded: gather_masters() assembles them (checkpoints, tests)."""

    BF16RS_MIN_BYTES = 4 << 20

    def __init__(self, model, group=None, bucket_bytes=256 * 1024, comm="auto", grad_comm="auto"):
        self.m = model
        self.group = group
        self.active = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.active else 1
        self.rank = dist.get_rank(group) if self.active else 0
        if grad_comm not in ("auto", "fp32", "bf16rs"):
            raise ValueError(f"grad_comm {grad_comm!r}")
        if grad_comm == "auto":
            per_layer = getattr(model, "fused_mode", None) is None and getattr(model, "W0f", None) is None
            big = model.grad_flat.numel() * 4 > self.BF16RS_MIN_BYTES
            force = os.environ.get("HPNN_DPX_FORCE", "0") == "1"  # the N > 1 path on one rank (tests)
            grad_comm = "bf16rs" if (self.active and (self.world > 1 or force) and per_layer and big) else "fp32"
        self.grad_comm = grad_comm
        self.sharded = set()
        if grad_comm == "bf16rs" and self.active and (self.world > 1 or os.environ.get("HPNN_DPX_FORCE", "0") == "1"):
            if getattr(model, "W0f", None) is not None or getattr(model, "fused_mode", None) is not None:
                raise ValueError("grad_comm='bf16rs' needs the per-layer path (fused=False)")
            self.sharded = {l for l in range(model.L) if model.Np[l] % self.world == 0}
        if self.active and self.world > 1 and self.rank == 0:
            # the exchange "auto" chose (bf16rs changes the numerics of large nets)
            print(f"data-parallel gradient exchange: {grad_comm}", file=sys.stderr, flush=True)
        self.buckets = self._plan(bucket_bytes)
        self.native = None
        self.dpx = None
        self.xar_inplace = False  # last fused xGMI step wrote its gradient in place
        on_gpu = getattr(model, "device", torch.device("cpu")).type == "cuda"
        if self.active and on_gpu and comm == "xar":
            from .comm import NativeComm
            self.native = NativeComm(group, device=model.device.index, rccl=False)
        elif self.active and on_gpu and (comm == "native" or (comm == "auto" and dist.get_backend(group) == "nccl")):
            from .comm import NativeComm
            self.native = NativeComm(group, device=model.device.index)
        # fused MNIST modes on the xGMI communicator: a second one whose protocol runs inside
        # the first-layer gradient launch (BPlan.xchg_step: front + ONE launch for G0, its
        # reduction, the exchange and every step -- the single-GPU step's launch count)
        self.xar_k = 0
        if (self.native is not None and self.native.xar and _XAR_G0 and getattr(model, "fused_mode", None) in ("x", "t")
                and model.grad_flat.numel() * 4 <= self.native.xar_max):
            self.xar_k = self.native.attach_xar_kernel(model.grad_flat.numel() * 4)
            if self.xar_k:
                # the in-kernel exchange itself on the real links (a known pattern through the
                # G0 launch's own barrier / peer-sum code, both one- and two-shot), agreed by
                # every rank before a gradient goes through it; -1: the shape never takes it
                rc = model.plan.xchg_self_test(self.xar_k, torch.cuda.current_stream().cuda_stream)
                if rc not in (0, -1):
                    print(f"rank {self.rank}: in-kernel xGMI exchange self-test failed ({rc}); "
                          f"using the all-reduce launch", flush=True)
                if not self.all_ok(rc in (0, -1)):
                    self.xar_k = 0
        # HPNN_DPX_FORCE=1 (tests): the native exchange even on one rank (with HPNN_DPX_SHARD1=1
        # its BF16 reduce-scatter path too), so a one-GPU box runs its kernels
        dpx_one = os.environ.get("HPNN_DPX_FORCE", "0") == "1"
        if self.native is not None and self.native.h and (self.world > 1 or dpx_one):
            # the library's data-parallel step (csrc/dist/dp_exchange.h): per-layer exchange on
            # the communicator's side stream, overlapped with the backward; BF16 reduce-scatter
            # + sharded step + BF16 all-gather for grad_comm="bf16rs" (no per-step allocation)
            from .._lib import native as _native
            self.dpx = _native().DpExchange(model.plan, self.native.h, 1 if self.sharded else 0)
            if self.sharded:
                self.sharded = {l for l in range(model.L) if self.dpx.sharded(l)}

    def _plan(self, bucket_bytes):
        """Group layers (descending = production order) into contiguous buckets."""
        m = self.m
        buckets, cur, cur_bytes = [], [], 0
        for l in range(m.L - 1, -1, -1):
            cur.append(l)
            cur_bytes += m.G[l].numel() * 4
            # the fused path produces [G1 | G2] long before G0 (whose GEMM is the last
            # backward kernel): close the bucket there so its all-reduce overlaps that GEMM
            fused_cut = getattr(m, "fused", False) and l == 1
            if cur_bytes >= bucket_bytes or l == 0 or fused_cut:
                buckets.append(cur)
                cur, cur_bytes = [], 0
        return buckets

    def broadcast_parameters(self, src=0):
        """Make every replica start from rank src's weights (reference: MPI_Bcast at
        generate/load, ann.c:709-763)."""
        if self.world == 1:
            return
        for l in range(self.m.L):
            for t in (self.m.W32[l], self.m.V32[l]):
                if t is None:
                    continue
                if self.native is not None and self.native.h:
                    self.native.broadcast(t, root=dist.get_group_rank(self.group, src) if self.group else src)
                elif dist.get_backend(self.group) != "nccl" and t.is_cuda:
                    c = t.cpu()
                    dist.broadcast(c, src, group=self.group)
                    t.copy_(c)
                else:
                    dist.broadcast(t, src, group=self.group)
        self.m.refresh_bf16()

    def check(self):
        """failure detection: raise if the communicator reported an asynchronous error"""
        if self.native is not None:
            self.native.check()

    def all_ok(self, ok=True):
        """every rank agrees on a status (replaces the reference's MPI bail-out)"""
        if not self.active:
            return bool(ok)
        if self.native is not None:
            return self.native.all_ok(ok)
        dev = self.m.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(t.item())

    def weights_consistent(self):
        """True when every replica holds bitwise-identical weights (digest all-gathered):
        catches an exchange that completed in time but summed the wrong data.  BF16 copies
        only when the sharded optimizer keeps the FP32 masters split over the ranks."""
        d = self.m.weights_digest(1 if self.sharded else 3)
        if not self.active or self.world == 1:
            return True
        dev = self.m.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        mine = torch.tensor([d & 0xFFFFFFFF, d >> 32], dtype=torch.int64, device=dev)
        every = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(every, mine, group=self.group)
        return all(torch.equal(e, every[0]) for e in every)

    def _bucket_view(self, layers):
        lo, hi = min(layers), max(layers)
        m = self.m
        start = m.G[lo].data_ptr() - m.grad_flat.data_ptr()
        end = m.G[hi].data_ptr() - m.grad_flat.data_ptr() + m.G[hi].numel() * 4
        return m.grad_flat[start // 4:end // 4]

    def _fused_xgmi_step(self, X, labels, T, n_valid, lr, alpha):
        """MNIST fused path on the xGMI all-reduce: 3 launches per step -- fused front, G0
        GEMM (+ first [G1|G2] reduction pass on its tail workgroups), ONE all-reduce whose
        copy-in phase also sums the local split-K slabs of G0 and the [G1|G2] groups and
        which then applies every layer's update to the reduced gradients"""
        m = self.m
        scale = 1.0 / (n_valid * self.world)
        if self.xar_k and m.plan.xchg_step(*m._x(X), *m._tgt(labels, T), int(n_valid), float(lr), float(alpha),
                                           float(scale), self.xar_k, torch.cuda.current_stream().cuda_stream):
            self.xar_inplace = "kernel"
            return
        segs = m.grads_slabs(X, labels, T, n_valid, dst=self.native.xar_local() if _XAR_UPD and _XAR_LOCAL else None)
        layers = [(m.W32[l], m.V32[l], m.Wb[l], m.Wt[l], m.W0f if l == 0 else None) for l in range(m.L)]
        self.xar_inplace = "buffer" if not segs else False
        if not segs:
            # the G0 launch wrote the reduced local gradient straight into the all-reduce's
            # buffer: barrier, peer sums and every layer's step, no copy-in
            self.native.reduce_local_update(m.grad_flat, layers, lr, alpha, scale, m.momentum)
        elif _XAR_UPD:
            # exchange + every layer's optimizer step in ONE launch (the update kernel and
            # its launch gap leave the data-parallel step)
            self.native.all_reduce_slabs_update(m.grad_flat, segs, layers, lr, alpha, scale, m.momentum)
        else:
            self.native.all_reduce_slabs(m.grad_flat, segs)
            m.update_all(lr, alpha, scale)

    def train_step(self, X, labels=None, T=None, n_valid=None, lr=0.01, alpha=0.2):
        m = self.m
        n_valid = m.Bp if n_valid is None else n_valid
        if not self.active:
            return m.train_step(X, labels=labels, T=T, n_valid=n_valid, lr=lr, alpha=alpha)
        if (self.native is not None and self.native.xar and getattr(m, "fused_mode", None) in ("x", "t")
                and m.grad_flat.numel() * 4 <= self.native.xar_max):
            return self._fused_xgmi_step(X, labels, T, n_valid, lr, alpha)
        if self.dpx is not None:
            self.dpx.step(*m._x(X), *m._tgt(labels, T), int(n_valid), int(n_valid) * self.world, float(lr),
                          float(alpha), torch.cuda.current_stream().cuda_stream)
            return
        works = []
        done = set()

        def ready(l):
            done.add(l)
            for b in self.buckets:
                if b[-1] == l and all(x in done for x in b):
                    if self.native is not None:
                        self.native.all_reduce_async(self._bucket_view(b))
                    else:
                        works.append(dist.all_reduce(self._bucket_view(b), group=self.group, async_op=True))

        if self.sharded:
            return self._sharded_step(X, labels, T, n_valid, lr, alpha)
        m.backward_grads(X, labels=labels, T=T, n_valid=n_valid, reduce=True, on_ready=ready)
        scale = 1.0 / (n_valid * self.world)
        if self.native is not None:
            self.native.join()
        for w in works:
            w.wait()
        m.update_all(lr, alpha, scale)  # every layer from the reduced buckets


    # ------------------------------------------------------------ bf16rs (sharded) step
    def _rs(self, out, inp):
        """reduce-scatter of inp (rows stacked by rank) into out"""
        if self.native is not None and self.native.h:
            self.native.reduce_scatter(out, inp)
        elif dist.get_backend(self.group) == "nccl":
            dist.reduce_scatter_tensor(out, inp, group=self.group)
        else:  # gloo: the sum, then this rank's rows
            t = inp.float()
            dist.all_reduce(t, group=self.group)
            out.copy_(t.view(self.world, *out.shape)[self.rank])

    def _ag(self, out, inp):
        """all-gather of inp (this rank's rows) into out (rows stacked by rank)"""
        if self.native is not None and self.native.h:
            self.native.all_gather(out, inp)
        elif dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(out, inp.contiguous(), group=self.group)
        else:
            parts = [torch.empty_like(inp) for _ in range(self.world)]
            dist.all_gather(parts, inp.contiguous(), group=self.group)
            out.copy_(torch.cat(parts))

    def _sharded_step(self, X, labels, T, n_valid, lr, alpha):
        """bf16rs over torch.distributed (gloo / CPU tests: the emulation of the native
        DpExchange step's math; GPU runs with the native communicator take self.dpx)"""
        m, W = self.m, self.world
        m.backward_grads(X, labels=labels, T=T, n_valid=n_valid, reduce=True)
        scale = 1.0 / (n_valid * W)
        full = [l for l in range(m.L) if l not in self.sharded]
        if full:  # layers whose rows do not split evenly: the FP32 all-reduce
            for l in full:
                if self.native is not None and self.native.h:
                    self.native.all_reduce(m.G[l])
                else:
                    dist.all_reduce(m.G[l], group=self.group)
                m.update_layer(l, lr, alpha, scale, from_G=True)
        for l in sorted(self.sharded):
            N, K = m.Np[l], m.Kp[l]
            rp = N // W
            r0 = self.rank * rp
            g16 = m.G[l].to(torch.bfloat16)
            mine = torch.empty(rp, K, dtype=torch.bfloat16, device=g16.device)
            self._rs(mine, g16)
            Wt_scratch = torch.empty(K, rp, dtype=torch.bfloat16, device=g16.device)
            wb_rows = torch.empty(rp, K, dtype=torch.bfloat16, device=g16.device)
            ops.sgd_update(m.W32[l][r0:r0 + rp], None if m.V32[l] is None else m.V32[l][r0:r0 + rp],
                           mine.float(), wb_rows, Wt_scratch, lr, alpha, scale, m.momentum)
            self._ag(m.Wb[l], wb_rows)
            m.Wt[l].copy_(m.Wb[l].t())

    def gather_masters(self):
        """bf16rs: the FP32 master weights / momentum rows of every rank onto every rank"""
        m = self.m
        if self.dpx is not None:
            self.dpx.gather_masters(torch.cuda.current_stream().cuda_stream)
            return
        for l in sorted(self.sharded):
            rp = m.Np[l] // self.world
            r0 = self.rank * rp
            for t in (m.W32[l], m.V32[l]):
                if t is not None:
                    self._ag(t, t[r0:r0 + rp].clone())


def init_from_env(backend=None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torchrun) if needed.
    Returns (rank, world_size, local_rank)."""
    import os
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # HPNN_DP_FORCE=1: build the process group even for one rank, so the bucketed
    # all-reduce path (RCCL on a GPU) can be exercised on a single-GPU box
    force = os.environ.get("HPNN_DP_FORCE", "0") == "1" and "MASTER_ADDR" in os.environ
    if (ws > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, ws, local


def ops_available():
    return ops is not None
