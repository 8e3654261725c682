#!/usr/bin/env python3
"""Per-call time of the xGMI all-reduce (csrc/dist/xgmi_ar.hip) with W processes.

On a 1-GPU box all ranks share device 0, so this measures the protocol cost (fine-grained
flag barriers, copy-in, fixed-order sums) over local HBM, not xGMI link bandwidth.
usage: python scripts/xar_bench.py [--world 2] [--mode 0|1|2] [--floats 109568] [--iters 200]"""
import argparse
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, a, port, q):
    os.environ["HPNN_XAR_MODE"] = str(a.mode)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from hpnn_amd._lib import native
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=a.world)
    n = native()
    x = n.xar_create(rank, a.world, 4 << 20)
    h = torch.tensor(list(n.xar_handles(x)), dtype=torch.uint8)
    allh = torch.zeros(a.world * n.XAR_HANDLE_BYTES, dtype=torch.uint8)
    dist.all_gather_into_tensor(allh, h)
    n.xar_open(x, bytes(allh.tolist()))
    buf = torch.randn(a.floats, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(20):
        n.xar_all_reduce_f32(x, buf.data_ptr(), buf.data_ptr(), a.floats, s)
    torch.cuda.synchronize()
    dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        n.xar_all_reduce_f32(x, buf.data_ptr(), buf.data_ptr(), a.floats, s)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    ok = n.xar_status(x) == 0
    dist.barrier()
    n.xar_destroy(x)
    q.put((rank, us, ok))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--floats", type=int, default=109568)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, a, port, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    print(f"world {a.world} mode {a.mode} floats {a.floats}: " +
          " ".join(f"r{r} {us:.1f}us{'' if ok else ' TIMEOUT'}" for r, us, ok in res))


if __name__ == "__main__":
    main()
