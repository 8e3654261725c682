"""Race detection for the GPU training step by bitwise determinism.

Every reduction of the batched engine is deterministic by construction (split-K slabs
summed in a fixed order, no floating-point atomics on weights or gradients; only the
loss / hit statistics use atomics).  So two runs of the same steps from the same state
on the same inputs must produce bit-identical weights and momentum: any difference means
a kernel reads LDS / global memory it does not own yet (missing barrier, wrong waitcnt,
overlapping ring slots) -- a data race.  GPU sanitizers and xnack are unavailable on
the target pool, so this is the race detector the tests and users run
(`python -m hpnn_amd.utils.racecheck`).  The reference has none."""
import argparse

import torch


def _state(m):
    return [t.clone() for t in m.W32] + [t.clone() for t in m.V32 if t is not None]


def check(make_model, make_batch, steps=5, repeats=3, lr=0.05, alpha=0.2):
    """make_model() -> fresh MLP, make_batch(model, i) -> (X, labels).  Returns the list
    of mismatching tensor indices per repeat ([] everywhere = deterministic)."""
    ref = None
    bad = []
    for r in range(repeats):
        m = make_model()
        for i in range(steps):
            X, lab = make_batch(m, i)
            m.train_step(X, labels=lab, lr=lr, alpha=alpha)
        torch.cuda.synchronize()
        st = _state(m)
        if ref is None:
            ref = st
            continue
        bad.append([j for j, (a, b) in enumerate(zip(ref, st)) if not torch.equal(a, b)])
    return bad


def main():
    from hpnn_amd.models import MLP
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--sizes", default="784,128,64,10")
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--fused", default="auto", choices=["auto", "x", "mid", "none"])
    a = ap.parse_args()
    sizes = [int(s) for s in a.sizes.split(",")]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    Xr = [torch.rand(a.batch, sizes[0], device=dev, generator=g) for _ in range(2)]
    L = [torch.randint(0, sizes[-1], (a.batch,), device=dev, generator=g, dtype=torch.int32) for _ in range(2)]
    fused = {"auto": None, "none": False}.get(a.fused, a.fused)

    def mk():
        return MLP(sizes, "SNN", batch=a.batch, device=dev, momentum=True, seed=3, fused=fused)

    cache = {}

    def batch(m, i):
        k = (id(m), i % 2)
        if k not in cache:
            cache[k] = m.prepare_input(Xr[i % 2])
        return cache[k], L[i % 2]

    bad = check(mk, batch, a.steps, a.repeats)
    ok = all(not b for b in bad)
    print(f"racecheck sizes={sizes} batch={a.batch} fused={a.fused}: {'deterministic' if ok else f'MISMATCH {bad}'}")
    raise SystemExit(0 if ok else 1)


if __name__ == "__main__":
    main()
