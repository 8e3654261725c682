"""Random kernel generator: ``python -m hpnn_amd.utils.gen_ann N_IN H1 ... N_OUT``.

Counterpart of the reference's ``scripts/gen_ann.bash``: writes a
``kernel.opt`` (grammar in :mod:`hpnn_amd.utils.formats`) to stdout or ``-o FILE``,
named ``auto``, with every weight ``2 (u - 0.5) / sqrt(n)`` where ``u`` is uniform in
[0, 1) and ``n`` is the neuron count of the layer being written -- the reference
script's scale (gen_ann.bash:45-48; note it divides by the layer's OUTPUT width, not
the fan-in the library's own ``[init] generate`` uses), printed ``%7.5f``.

Differences: the reference draws its digits from ``/dev/urandom`` through
``hexdump -d`` (so ``u`` only spans [0, 0.65535]: its weights are biased negative);
here ``u`` comes from a seedable generator (``--seed``; default: OS entropy) and is
uniform, so generated kernels are reproducible and zero-mean.  ``--fan-in`` switches
the scale to ``1/sqrt(fan_in)``.
"""
import argparse
import sys

import numpy as np


def generate(sizes, seed=None, fan_in=False):
    """List of weight matrices [N_l x N_{l-1}] (FP64) for the layer sizes ``sizes``."""
    if len(sizes) < 3:
        raise ValueError("need num_input, at least one hidden layer and num_output")
    if any(int(s) < 1 for s in sizes):
        raise ValueError("layer sizes must be >= 1")
    rng = np.random.default_rng(seed)
    ws = []
    for prev, n in zip(sizes[:-1], sizes[1:]):
        u = rng.random((int(n), int(prev)))
        ws.append(2.0 * (u - 0.5) / np.sqrt(prev if fan_in else n))
    return ws


def write(f, weights, name="auto"):
    sizes = [weights[0].shape[1]] + [w.shape[0] for w in weights]
    f.write(f"[name] {name}\n[param] " + " ".join(map(str, sizes)) + "\n")
    f.write(f"[input] {sizes[0]}\n")
    for l, W in enumerate(weights):
        last = l == len(weights) - 1
        f.write(f"[output] {W.shape[0]}\n" if last else f"[hidden {l + 1}] {W.shape[0]}\n")
        for j, row in enumerate(W):
            f.write(f"[neuron {j + 1}] {W.shape[1]}\n")
            f.write("".join("%7.5f " % v for v in row) + "\n")


def main(argv=None):
    p = argparse.ArgumentParser(prog="gen_ann", description="random kernel.opt generator")
    p.add_argument("sizes", nargs="+", type=int, help="num_input num_hid1 ... num_hidN num_output")
    p.add_argument("-o", "--output", default="-", help="output file (default stdout)")
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--fan-in", action="store_true", help="scale by 1/sqrt(fan_in)")
    p.add_argument("--name", default="auto")
    a = p.parse_args(argv)
    try:
        ws = generate(a.sizes, a.seed, a.fan_in)
    except ValueError as e:
        print(f"ERROR: {e}", file=sys.stderr)
        return 1
    if a.output == "-":
        write(sys.stdout, ws, a.name)
    else:
        with open(a.output, "w") as f:
            write(f, ws, a.name)
    return 0


if __name__ == "__main__":
    sys.exit(main())
