"""Training monitor: ASCII plot of the per-pass accuracy a tutorial run logs.

The reference's MNIST tutorial starts a ``watch`` loop that greps the ``run_nn`` logs
into a file and renders it with gnuplot's dumb terminal (``tutorials/mnist/tutorial.bash:
138-174``, ``tutorials/mnist/plot.gnuplot:1-6``).  Here the tutorials already write one
``pass accuracy[%] [loss=...]`` line per pass to ``WORK/raw``
(``tutorials/mnist/tutorial.sh``, ``tutorials/rruff/tutorial.sh``); this module renders that
file as a text chart, once or refreshed while training runs (``--follow``), with no gnuplot.

    python -m hpnn_amd.utils.monitor mnist_run/raw            # one chart
    python -m hpnn_amd.utils.monitor mnist_run/raw --follow 5 # redraw every 5 s
"""
import argparse
import re
import sys
import time

_LOSS = re.compile(r"loss=([-+0-9.eE]+)")


def read_raw(path):
    """-> list of (pass, accuracy, loss or None) from a tutorial ``raw`` file; lines that
    do not parse (a pass still being written, a failed run_nn) are skipped"""
    rows = []
    try:
        with open(path) as f:
            lines = f.read().splitlines()
    except FileNotFoundError:
        return rows
    for ln in lines:
        parts = ln.split()
        if len(parts) < 2:
            continue
        try:
            p, acc = int(parts[0]), float(parts[1])
        except ValueError:
            continue
        m = _LOSS.search(ln)
        rows.append((p, acc, float(m.group(1)) if m else None))
    return rows


def render(rows, width=60, height=15, title="test accuracy [%] per pass"):
    """Text chart of accuracy (y, 0-100 scaled to the data) against pass (x)."""
    if not rows:
        return f"{title}\n(no data yet)\n"
    width, height = max(width, 10), max(height, 4)
    xs = [r[0] for r in rows]
    ys = [r[1] for r in rows]
    x0, x1 = min(xs), max(xs)
    lo, hi = min(ys), max(ys)
    if hi - lo < 1e-9:
        lo, hi = max(0.0, lo - 1.0), min(100.0, hi + 1.0)
        if hi <= lo:
            hi = lo + 1.0
    grid = [[" "] * width for _ in range(height)]
    for x, y in zip(xs, ys):
        c = 0 if x1 == x0 else round((x - x0) * (width - 1) / (x1 - x0))
        r = round((hi - y) * (height - 1) / (hi - lo))
        grid[r][c] = "*"
    out = [title]
    for i, row in enumerate(grid):
        label = hi - i * (hi - lo) / (height - 1)
        out.append(f"{label:7.2f} |" + "".join(row))
    out.append(" " * 8 + "+" + "-" * width)
    out.append(" " * 9 + f"{x0:<{width // 2}d}{x1:>{width - width // 2}d}")
    last = rows[-1]
    tail = f"pass {last[0]}: {last[1]:.2f} %"
    if last[2] is not None:
        tail += f"  loss {last[2]:.6g}"
    out.append(tail + f"  (best {max(ys):.2f} % at pass {xs[ys.index(max(ys))]})")
    return "\n".join(out) + "\n"


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("raw", help="tutorial raw file (pass accuracy [loss=...] per line)")
    ap.add_argument("--width", type=int, default=60)
    ap.add_argument("--height", type=int, default=15)
    ap.add_argument("--follow", type=float, default=0.0, help="redraw every N seconds until interrupted")
    ap.add_argument("--count", type=int, default=0, help="with --follow: stop after N redraws (0 = forever)")
    a = ap.parse_args(argv)
    n = 0
    while True:
        chart = render(read_raw(a.raw), a.width, a.height)
        if a.follow > 0:
            sys.stdout.write("\x1b[2J\x1b[H")
        sys.stdout.write(chart)
        sys.stdout.flush()
        n += 1
        if a.follow <= 0 or (a.count and n >= a.count):
            return 0
        time.sleep(a.follow)


if __name__ == "__main__":
    sys.exit(main())
