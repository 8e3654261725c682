"""libhpnn text formats (conf, sample, kernel.opt) in Python.

Grammars (docs/FORMATS.md; reference ann.c:770-857 / libhpnn.c:658-937 / 1070-1145):

  conf      [name] x / [type] ANN|SNN|LNN / [init] generate|<kernel file> / [seed] n /
            [input] n / [hidden] h1 h2 ... / [output] n / [train] BP|BPM|CG|SPLX /
            [sample_dir] d / [test_dir] d   (+ optional [mode] [batch] [epochs] [dtype]
            [device] [lr] [momentum])
  sample    [input] N \\n v1 ... vN \\n [output] M  #comment \\n t1 ... tM
  kernel    [name] / [param] n_in h.. n_out / [input] n_in / per layer [hidden i] N or
            [output] N, then per neuron "[neuron j] M" + one line of M weights (%17.15f)

These mirror the C reader/writer in csrc/core so Python tools and tests can produce and
check files without the native library.
"""
import re

import numpy as np


def write_sample(path, x, t, comment=None):
    with open(path, "w") as f:
        f.write(f"[input] {len(x)}\n")
        f.write(" ".join(f"{v:7.5f}" for v in x) + "\n")
        f.write(f"[output] {len(t)}" + (f"  #{comment}" if comment is not None else "") + "\n")
        f.write(" ".join(f"{v:.1f}" for v in t) + "\n")


def read_sample(path):
    x = t = None
    with open(path) as f:
        lines = f.read().splitlines()
    i = 0
    while i < len(lines):
        ln = lines[i]
        m = re.search(r"\[(input|output)[^\]]*\]\s*(\d+)", ln)
        if m:
            n = int(m.group(2))
            vals = []
            i += 1
            while len(vals) < n and i < len(lines):
                vals += [float(v) for v in lines[i].split()]
                i += 1
            arr = np.array(vals[:n], dtype=np.float64)
            if m.group(1) == "input":
                x = arr
            else:
                t = arr
            continue
        i += 1
    if x is None or t is None:
        raise ValueError(f"malformed sample {path}")
    return x, t


def write_conf(path, name="nn", type="SNN", init="generate", seed=0, inputs=None, hiddens=(), outputs=None,
               train="BP", sample_dir="./samples", test_dir="./tests", **extra):
    with open(path, "w") as f:
        f.write("# libhpnn configuration\n")
        f.write(f"[name] {name}\n[type] {type}\n[init] {init}\n[seed] {seed}\n")
        if inputs is not None:
            f.write(f"[input] {inputs}\n")
        if hiddens:
            f.write("[hidden] " + " ".join(str(h) for h in hiddens) + "\n")
        if outputs is not None:
            f.write(f"[output] {outputs}\n")
        f.write(f"[train] {train}\n[sample_dir] {sample_dir}\n[test_dir] {test_dir}\n")
        for k, v in extra.items():
            f.write(f"[{k}] {v}\n")


def read_conf(path):
    out = {}
    with open(path) as f:
        for ln in f:
            m = re.match(r"\s*\[([a-z_]+)[^\]]*\]\s*(.*)", ln)
            if not m:
                continue
            k, v = m.group(1), m.group(2).split("#")[0].strip()
            k = {"inputs": "input", "hiddens": "hidden", "outputs": "output"}.get(k, k)
            if k == "hidden":
                out[k] = [int(x) for x in v.split()]
            elif k in ("input", "output", "seed", "batch", "epochs"):
                out[k] = int(v)
            else:
                out[k] = v
    return out


def write_kernel(path, weights, name="noname", exact=False):
    fmt = "{:.17g}" if exact else "{:17.15f}"
    sizes = [weights[0].shape[1]] + [w.shape[0] for w in weights]
    with open(path, "w") as f:
        f.write(f"[name] {name}\n")
        f.write("[param] " + " ".join(str(s) for s in sizes) + "\n")
        f.write(f"[input] {sizes[0]}\n")
        for l, W in enumerate(weights):
            W = np.asarray(W, dtype=np.float64)
            last = l == len(weights) - 1
            f.write(f"[output] {W.shape[0]}\n" if last else f"[hidden {l + 1}] {W.shape[0]}\n")
            for j in range(W.shape[0]):
                f.write(f"[neuron {j + 1}] {W.shape[1]}\n")
                f.write(" ".join(fmt.format(v) for v in W[j]) + "\n")


def read_kernel(path):
    name, blocks, cur, rows = "noname", [], None, None
    with open(path) as f:
        lines = f.read().splitlines()
    i = 0
    pending = None
    while i < len(lines):
        ln = lines[i].strip()
        if ln.startswith("[name"):
            name = ln.split("]", 1)[1].strip()
        elif ln.startswith("[hidden") or ln.startswith("[output"):
            n = int(ln.split("]", 1)[1])
            cur = {"n": n, "rows": [None] * n}
            blocks.append(cur)
        elif ln.startswith("[neuron"):
            j = int(re.match(r"\[neuron\s+(\d+)", ln).group(1)) - 1
            m = int(ln.split("]", 1)[1])
            vals = []
            i += 1
            while len(vals) < m and i < len(lines):
                vals += [float(v) for v in lines[i].split()]
                i += 1
            cur["rows"][j] = vals[:m]
            continue
        i += 1
    del rows, pending
    weights = [np.array(b["rows"], dtype=np.float64) for b in blocks]
    return {"name": name, "weights": weights, "sizes": [weights[0].shape[1]] + [w.shape[0] for w in weights]}
