"""Diagnostics: where the fixed cost of a short timed region goes (driver-style K = 20).

Builds the MNIST bench step as bench.py does, settles the clock, then repeats the timed-region
pattern (synchronize, t0, replay one 20-step graph, synchronize, t1) and reports per repeat:
host wall time, GPU time between events recorded around the replay, and the gap between
them, plus variants: an idle gap of G us before the region (busy-wait on the host) and
back-to-back replays without a synchronize between them."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpnn_amd.models import MLP  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    m = MLP([784, 128, 64, 10], "SNN", batch=65536, device=dev, momentum=True, seed=10958)
    g = torch.Generator(device=dev).manual_seed(1234)
    Xs = [m.prepare_input(torch.randint(0, 256, (m.Bp, 784), device=dev, generator=g, dtype=torch.uint8))
          for _ in range(4)]
    Ls = [torch.randint(0, 10, (m.Bp,), device=dev, generator=g, dtype=torch.int32) for _ in range(4)]
    for i in range(3):
        m.train_step(Xs[i % 4], labels=Ls[i % 4])
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m.train_step(Xs[0], labels=Ls[0])
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(gr):
        for i in range(20):
            m.train_step(Xs[i % 4], labels=Ls[i % 4])
    g5 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g5):
        for i in range(5):
            m.train_step(Xs[i % 4], labels=Ls[i % 4])
    torch.cuda.synchronize()
    for _ in range(45):  # settle ~50 ms
        gr.replay()
    torch.cuda.synchronize()
    out = {}
    # bench.py's sequence before its clock: another graph (the W = 5 warmup), synchronize,
    # the statistics reset, synchronize
    rows = []
    for rep in range(8):
        g5.replay()
        torch.cuda.synchronize()
        m.reset_stats()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        gr.replay()
        b.record()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rows.append(((t1 - t0) * 1e3 / 20, a.elapsed_time(b) / 20))
    out["after_g5"] = rows
    for idle_us in (0, 100, 1000, 10000):
        rows = []
        for rep in range(8):
            torch.cuda.synchronize()
            t_end = time.perf_counter() + idle_us * 1e-6
            while time.perf_counter() < t_end:
                pass
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            a.record()
            gr.replay()
            b.record()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            rows.append(((t1 - t0) * 1e3 / 20, a.elapsed_time(b) / 20))
        out[f"idle{idle_us}us"] = rows
    # back to back: 10 replays, per-replay GPU time
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(11)]
    torch.cuda.synchronize()
    ev[0].record()
    for i in range(10):
        gr.replay()
        ev[i + 1].record()
    torch.cuda.synchronize()
    out["b2b_gpu_ms_per_step"] = [ev[i].elapsed_time(ev[i + 1]) / 20 for i in range(10)]
    for k, v in out.items():
        print(k, json.dumps([[round(x * 1e3, 2) for x in r] if isinstance(r, tuple) else round(r * 1e3, 2) for r in v]))


if __name__ == "__main__":
    main()
