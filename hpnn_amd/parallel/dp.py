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
import torch
import torch.distributed as dist

from .. import ops


class DataParallel:
    def __init__(self, model, group=None, bucket_bytes=256 * 1024):
        self.m = model
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.buckets = self._plan(bucket_bytes)

    def _plan(self, bucket_bytes):
        """Group layers (descending = production order) into contiguous buckets."""
        m = self.m
        buckets, cur, cur_bytes = [], [], 0
        for l in range(m.L - 1, -1, -1):
            cur.append(l)
            cur_bytes += m.G[l].numel() * 4
            if cur_bytes >= bucket_bytes or l == 0:
                buckets.append(cur)
                cur, cur_bytes = [], 0
        return buckets

    def broadcast_parameters(self, src=0):
        """Make every replica start from rank src's weights (reference: MPI_Bcast at
        generate/load, ann.c:709-763)."""
        if self.world == 1:
            return
        for l in range(self.m.L):
            dist.broadcast(self.m.W32[l], src, group=self.group)
            if self.m.V32[l] is not None:
                dist.broadcast(self.m.V32[l], src, group=self.group)
        self.m.refresh_bf16()

    def _bucket_view(self, layers):
        lo, hi = min(layers), max(layers)
        m = self.m
        start = m.G[lo].data_ptr() - m.grad_flat.data_ptr()
        end = m.G[hi].data_ptr() - m.grad_flat.data_ptr() + m.G[hi].numel() * 4
        return m.grad_flat[start // 4:end // 4]

    def train_step(self, X, labels=None, T=None, n_valid=None, lr=0.01, alpha=0.2):
        m = self.m
        n_valid = m.Bp if n_valid is None else n_valid
        if self.world == 1:
            return m.train_step(X, labels=labels, T=T, n_valid=n_valid, lr=lr, alpha=alpha)
        works = []
        done = set()

        def ready(l):
            done.add(l)
            for b in self.buckets:
                if b[-1] == l and all(x in done for x in b):
                    works.append(dist.all_reduce(self._bucket_view(b), group=self.group, async_op=True))

        m.backward_grads(X, labels=labels, T=T, n_valid=n_valid, reduce=True, on_ready=ready)
        scale = 1.0 / (n_valid * self.world)
        for w in works:
            w.wait()
        for l in range(m.L):
            m.update_layer(l, lr, alpha, scale, from_G=True)


def init_from_env(backend=None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torchrun) if needed.
    Returns (rank, world_size, local_rank)."""
    import os
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1 and not dist.is_initialized():
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
