"""Native RCCL communicator for the data-parallel hot path (libhpnn comm layer).

torch.distributed (backend "nccl" = RCCL on ROCm) owns the process group: rendezvous,
rank / world size, barriers and the one-time bootstrap.  The per-step gradient
all-reduce goes through libhpnn's own RCCL communicator instead
(include/libhpnn/comm.h, csrc/dist/comm.cpp): one C call per bucket, issued on a
high-priority side stream that forks from the compute stream with a hipEvent and joins
back before the update.  Measured on one MI355X (single-rank group, MNIST step of
84 us): the same bucketed step through ProcessGroupNCCL ran at 144 us per step, its
per-collective host bookkeeping being of the order of a whole training step; the
native path keeps the host cost of a step at a few microseconds and is capturable in
a HIP graph.

The reference's equivalent is MPI_Allreduce / MPI_Allgather inline in every compute
function (src/ann.c, e.g. ann.c:1263, 1638).
"""
import os

import torch
import torch.distributed as dist

from .._lib import native

DT_F32, DT_F64, DT_BF16, DT_I32, DT_U8 = 0, 1, 2, 3, 4
OP_SUM, OP_MAX, OP_MIN = 0, 1, 2
ID_BYTES = 128

_DT = {torch.float32: DT_F32, torch.float64: DT_F64, torch.bfloat16: DT_BF16, torch.int32: DT_I32,
       torch.uint8: DT_U8}


def _xar_wanted(world):
    """one-shot xGMI all-reduce: all ranks on this node (torchrun's LOCAL_WORLD_SIZE), at
    most 8, and not disabled with HPNN_XAR=0"""
    if os.environ.get("HPNN_XAR", "1") == "0" or world > 8:
        return False
    return int(os.environ.get("LOCAL_WORLD_SIZE", "0")) == world


def _stream():
    return torch.cuda.current_stream().cuda_stream


class NativeComm:
    """One libhpnn RCCL communicator per process (this process' current GPU).

    Bootstrap: rank 0 of `group` creates the RCCL unique id, torch.distributed
    broadcasts it, every rank calls ncclCommInitRank through libhpnn."""

    def __init__(self, group=None, device=None, rccl=True):
        """rccl=False: no RCCL communicator, only the one-shot xGMI all-reduce (used to
        exercise the data-parallel step with several processes on ONE GPU, where RCCL
        refuses duplicate devices)"""
        if not dist.is_initialized():
            raise RuntimeError("NativeComm needs an initialised torch.distributed process group")
        n = native()
        self.h = 0
        self.xar = 0
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.cuda.current_device() if device is None else int(device)
        if not rccl:
            if self.world < 2 or not self._attach_xar(int(os.environ.get("HPNN_XAR_MAX_BYTES", str(4 << 20)))):
                raise RuntimeError("xGMI all-reduce unavailable")
            return
        uid = torch.zeros(ID_BYTES, dtype=torch.uint8)
        if self.rank == 0:
            uid = torch.tensor(list(n.comm_unique_id()), dtype=torch.uint8)
        src = dist.get_global_rank(group, 0) if group is not None else 0
        if dist.get_backend(group) == "nccl":
            t = uid.to(torch.device("cuda", self.device))
            dist.broadcast(t, src, group=group)
            uid = t.cpu()
        else:
            dist.broadcast(uid, src, group=group)
        self.h = n.comm_init_rank(bytes(uid.tolist()), self.world, self.rank, self.device)
        if not self.h:
            raise RuntimeError("ncclCommInitRank failed (see stderr)")
        self.xar = 0
        # HPNN_DP_FORCE=1 (one rank): attach it anyway, so the N > 1 step path (slab sums in
        # the all-reduce's copy-in, then the update) can be timed on a single-GPU box
        if (self.world > 1 or os.environ.get("HPNN_DP_FORCE", "0") == "1") and _xar_wanted(self.world):
            self._attach_xar(int(os.environ.get("HPNN_XAR_MAX_BYTES", str(4 << 20))))

    def _attach_xar(self, max_bytes):
        """one-shot xGMI all-reduce for the small gradient buckets (include/libhpnn/xar.h):
        every rank maps every peer's buffer (hipIpc handles exchanged over the process
        group); all ranks agree before it is used, else every rank stays on RCCL"""
        x = self._open_xar(max_bytes)
        if not x:
            return False
        self.xar = x
        self.xar_max = max_bytes
        if self.h:
            native().comm_set_xar(self.h, x, max_bytes)
        return True

    def attach_xar_kernel(self, max_bytes):
        """a second xGMI communicator whose protocol runs inside a compute kernel (the fused
        data-parallel first-layer gradient, BPlan.xchg_step); collective, like the first.
        Returns its handle, 0 when unavailable on some rank."""
        if not self.xar:
            return 0
        if not getattr(self, "xar_kernel", 0):
            self.xar_kernel = self._open_xar(max_bytes)
        return self.xar_kernel

    def _open_xar(self, max_bytes):
        n = native()
        x = n.xar_create(self.rank, self.world, max_bytes)
        ok = bool(x)
        nb = n.XAR_HANDLE_BYTES
        h = torch.zeros(nb, dtype=torch.uint8)
        if ok:
            try:
                h = torch.tensor(list(n.xar_handles(x)), dtype=torch.uint8)
            except RuntimeError:
                ok = False
        dev = torch.device("cuda", self.device) if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        allh = torch.zeros(self.world * nb, dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(allh, h.to(dev), group=self.group)
        if ok:
            try:
                n.xar_open(x, bytes(allh.cpu().tolist()))
            except RuntimeError:
                ok = False
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) == 1 and os.environ.get("HPNN_XAR_SELFTEST", "1") != "0":
            # every rank mapped every peer: check on the real links that each rank receives
            # exactly the known sums (a mapping / coherence fault shows here, not as silently
            # wrong gradients later), then agree; any failure sends every rank to RCCL
            rc = n.xar_self_test(x, _stream())
            if rc != 0:
                print(f"rank {self.rank}: xGMI all-reduce self-test failed ({rc}); using RCCL", flush=True)
            flag.fill_(1 if rc == 0 else 0)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) != 1:
            if x:
                n.xar_destroy(x)
            return 0
        return x

    # -- collectives on the current stream ------------------------------------------
    def all_reduce(self, t, op=OP_SUM):
        native().comm_all_reduce(self.h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], op, _stream())
        return t

    def broadcast(self, t, root=0):
        native().comm_broadcast(self.h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], root, _stream())
        return t

    def all_gather(self, out, inp):
        """out: world * inp.numel() elements, rank r's block at r * inp.numel()"""
        native().comm_all_gather(self.h, inp.data_ptr(), out.data_ptr(), inp.numel(), _DT[inp.dtype], _stream())
        return out

    def reduce_scatter(self, out, inp, op=OP_SUM):
        native().comm_reduce_scatter(self.h, inp.data_ptr(), out.data_ptr(), out.numel(), _DT[inp.dtype], op,
                                     _stream())
        return out

    # -- overlapped gradient buckets ------------------------------------------------
    def all_reduce_async(self, t):
        """sum all-reduce of t on the side stream, after the work already on the current
        stream; overlaps whatever is enqueued next until join()"""
        if not self.h:  # xGMI-only: in order on the current stream
            native().xar_all_reduce_f32(self.xar, t.data_ptr(), t.data_ptr(), t.numel(), _stream())
            return
        native().comm_all_reduce_async(self.h, t.data_ptr(), t.numel(), _DT[t.dtype], _stream())

    def join(self):
        if self.h:
            native().comm_join(self.h, _stream())

    @staticmethod
    def _segs(segs):
        """segments as (address, slab stride, S, n) -- the form BPlan.grads_slabs returns --
        or (tensor [S, >= n], S, n)"""
        return [s if len(s) == 4 else (s[0].data_ptr(), s[0].stride(0), s[1], s[2]) for s in segs]

    def all_reduce_slabs(self, out, segs):
        """out = sum over ranks of [seg_0 | seg_1 | ...] where segment j is the local sum of
        its S slabs of n floats: split-K reduction and exchange in ONE launch (xGMI
        all-reduce, include/libhpnn/xar.h), on the current stream"""
        native().xar_all_reduce_slabs_f32(self.xar, self._segs(segs), out.data_ptr(), _stream())
        return out

    def all_reduce_slabs_update(self, out, segs, layers, lr, alpha, scale, momentum):
        """all_reduce_slabs followed, in the same launch, by every layer's optimizer step
        on the reduced gradient (include/libhpnn/xar.h hpnn_xar_all_reduce_slabs_update_f32);
        layers: [(W32, V32 or None, Wbf, Wt, Wf or None)] tiling `out` in order"""
        def p(t):
            return 0 if t is None else t.data_ptr()
        native().xar_all_reduce_slabs_update_f32(
            self.xar, self._segs(segs), out.data_ptr(),
            [(p(w), p(v), p(wb), p(wt), p(wf), w.shape[0], w.shape[1]) for w, v, wb, wt, wf in layers],
            float(lr), float(alpha), float(scale), int(bool(momentum)), _stream())
        return out

    def xar_local(self):
        """(buffer address, selector address, half stride in floats) of the in-place form
        (include/libhpnn/xar.h hpnn_xar_local)"""
        if not hasattr(self, "_xar_local"):
            self._xar_local = native().xar_local(self.xar)
        return self._xar_local

    def reduce_local_update(self, out, layers, lr, alpha, scale, momentum):
        """the in-place all-reduce + step: this rank's contribution already sits in the
        buffer half xar_local() selects (written by the G0 launch)"""
        def p(t):
            return 0 if t is None else t.data_ptr()
        native().xar_reduce_local_update_f32(
            self.xar, sum(w.shape[0] * w.shape[1] for w, *_ in layers), out.data_ptr(),
            [(p(w), p(v), p(wb), p(wt), p(wf), w.shape[0], w.shape[1]) for w, v, wb, wt, wf in layers],
            float(lr), float(alpha), float(scale), int(bool(momentum)), _stream())
        return out

    # -- failure detection ----------------------------------------------------------
    def check(self):
        """raise if the communicator saw an asynchronous error (peer died, link down) or an
        xGMI all-reduce barrier timed out"""
        if not self.h:
            if self.xar and native().xar_status(self.xar) != 0:
                raise RuntimeError(f"xGMI all-reduce barrier timed out on rank {self.rank}")
            return
        if native().comm_check(self.h) != 0:
            native().comm_abort(self.h)
            raise RuntimeError(f"RCCL communicator failed on rank {self.rank}")

    def all_ok(self, ok=True):
        """MIN over ranks of ok (the collective replacement of the reference's MPI
        bail-out after a failed kernel load, ann.c:237-249)"""
        if not self.h:
            t = torch.tensor([1 if ok else 0], dtype=torch.int32)
            if dist.get_backend(self.group) == "nccl":
                t = t.cuda(self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
            return bool(t.item())
        return bool(native().comm_all_ok(self.h, 1 if ok else 0, _stream()))

    def xar_healthy(self):
        """False when an xGMI all-reduce barrier of this rank timed out"""
        return all(not x or native().xar_status(x) == 0 for x in (self.xar, getattr(self, "xar_kernel", 0)))

    def detach_xar(self):
        """stop using the xGMI all-reduce (every rank must call it: RCCL takes over).  The
        buffers stay mapped until close(): a peer may still be inside a timed-out call."""
        if self.xar and self.h:
            native().comm_set_xar(self.h, 0, 0)
        self._xar_detached = self.xar
        self.xar = 0
        self._xar_kernel_detached = getattr(self, "xar_kernel", 0)
        self.xar_kernel = 0

    def close(self):
        for a in ("_xar_detached", "_xar_kernel_detached", "xar_kernel"):
            if getattr(self, a, 0):
                native().xar_destroy(getattr(self, a))
                setattr(self, a, 0)
        if getattr(self, "xar", 0):
            if self.h:
                native().comm_set_xar(self.h, 0, 0)
            native().xar_destroy(self.xar)
            self.xar = 0
        if self.h:
            native().comm_destroy(self.h)
            self.h = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
