"""Synthetic stand-ins for the tutorials' datasets (no network here, so neither MNIST
nor the RRUFF powder-XRD database can be downloaded).

``rruff_records`` writes RRUFF-shaped record pairs ``DIR/dif/NAME`` + ``DIR/raw/NAME``
that ``bin/pdif`` (the reference's ``tutorials/ann/prepare_dif.c``) turns into sample
files.  Each record belongs to one of a few space groups; the raw pattern is a sum of
Gaussian peaks whose 2-theta positions are a fixed function of the group plus jitter,
so the groups are learnable.  MNIST-shaped samples come from ``pmnist -g``.
"""
import os

import numpy as np

# (international number, Hermann-Mauguin symbol) -- symbols from the pdif table
GROUPS = [(2, "P-1"), (14, "P2_1/c"), (15, "C2/c"), (62, "Pnma"), (141, "I4_1/amd"),
          (154, "P3_221"), (166, "R-3m"), (194, "P6_3/mmc"), (225, "Fm-3m"), (227, "Fd-3m")]

_DIF = """      Synthetic   {name}
      Sample: T = {temp} K
      CELL PARAMETERS:    {a:.4f}    {a:.4f}    {c:.4f}   90.000   90.000  120.000
      SPACE GROUP: {sg}
               ATOM         X         Y         Z     OCCUPANCY  ISO(B)
                Si      0.4697    0.0000    0.0000    1.0000    0.5000
                 O      0.4135    0.2669    0.1191    1.0000    0.8000

            X-RAY WAVELENGTH:     1.541838
               2-THETA      INTENSITY    D-SPACING   H   K   L
{peaks}"""


def rruff_records(root, n, seed=0, groups=None, step=0.02):
    """Write ``n`` synthetic records under ``root/dif`` and ``root/raw``; returns the
    list of (name, space-group number)."""
    groups = GROUPS if groups is None else groups
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, "dif"), exist_ok=True)
    os.makedirs(os.path.join(root, "raw"), exist_ok=True)
    # per-group peak positions (degrees) and relative heights
    proto = []
    for g in range(len(groups)):
        r = np.random.default_rng(1000 + g)
        k = int(r.integers(4, 9))
        proto.append((np.sort(r.uniform(8, 85, k)), r.uniform(0.2, 1.0, k)))
    theta = np.arange(5.0, 90.0, step)
    out = []
    for i in range(n):
        g = int(rng.integers(len(groups)))
        num, sym = groups[g]
        pos, hgt = proto[g]
        pos = pos + rng.normal(0, 0.15, pos.size)
        hgt = hgt * rng.uniform(0.8, 1.2, hgt.size)
        y = 5.0 + rng.uniform(0, 2, theta.size)
        for p, h in zip(pos, hgt):
            y += 1000.0 * h * np.exp(-0.5 * ((theta - p) / 0.12) ** 2)
        name = f"S{i:06d}"
        peaks = "".join(f"{p:22.2f}{100 * h / hgt.max():14.2f}{1.5418 / (2 * np.sin(np.radians(p / 2))):15.4f}"
                        f"   1   0   0\n" for p, h in zip(pos, hgt))
        with open(os.path.join(root, "dif", name), "w") as f:
            f.write(_DIF.format(name=name, temp=f"{rng.uniform(250, 350):.1f}", a=rng.uniform(4, 6),
                                c=rng.uniform(5, 7), sg=sym, peaks=peaks))
        with open(os.path.join(root, "raw", name), "w") as f:
            f.write("##NAMES=synthetic\n##END=\n")
            f.write("".join(f"{t:.2f}, {v:.2f}\n" for t, v in zip(theta, y)))
        out.append((name, num))
    return out


def main(argv=None):
    import argparse
    p = argparse.ArgumentParser(prog="synth_rruff", description="synthetic RRUFF DIF+raw records")
    p.add_argument("root")
    p.add_argument("-n", type=int, default=200)
    p.add_argument("--seed", type=int, default=0)
    a = p.parse_args(argv)
    recs = rruff_records(a.root, a.n, a.seed)
    print(f"# wrote {len(recs)} synthetic records to {a.root}/dif and {a.root}/raw")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
