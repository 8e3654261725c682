"""Auxiliary tools on the CPU: the random kernel generator (reference
scripts/gen_ann.bash), the synthetic dataset writers and the two tutorials
(reference tutorials/mnist/tutorial.bash, tutorials/ann/tutorial.bash) end to end
on the FP64 CPU engine with tiny synthetic data."""
import os
import subprocess
import sys

import numpy as np
import pytest

from hpnn_amd.utils import formats, gen_ann

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


def _env():
    e = dict(os.environ)
    e["HPNN_FORCE_CPU"] = "1"
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    return e


def test_gen_ann_grammar_and_scale(tmp_path):
    p = tmp_path / "kernel.opt"
    r = subprocess.run([sys.executable, "-m", "hpnn_amd.utils.gen_ann", "20", "16", "8", "4", "--seed", "3",
                        "-o", str(p)], env=_env(), capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    lines = p.read_text().splitlines()
    assert lines[:4] == ["[name] auto", "[param] 20 16 8 4", "[input] 20", "[hidden 1] 16"]
    k = formats.read_kernel(str(p))
    assert k["sizes"] == [20, 16, 8, 4]
    ref = gen_ann.generate([20, 16, 8, 4], seed=3)
    for a, b, n in zip(k["weights"], ref, (16, 8, 4)):
        assert np.abs(a - b).max() <= 5e-6          # %7.5f
        assert np.abs(a).max() <= 1 / np.sqrt(n)    # 2(u-0.5)/sqrt(n_layer)
    assert subprocess.run([sys.executable, "-m", "hpnn_amd.utils.gen_ann", "3", "2"], env=_env(),
                          capture_output=True).returncode == 1


def test_gen_ann_kernel_loads_in_runtime(tmp_path):
    """a generated kernel is accepted by the C runtime ([init] FILE) and evaluated by run_nn"""
    d = tmp_path
    (d / "tests").mkdir()
    rng = np.random.default_rng(0)
    for i in range(5):
        t = np.zeros(3)
        t[i % 3] = 1
        formats.write_sample(str(d / "tests" / f"t{i}"), rng.uniform(-1, 1, 6), t)
    with open(d / "kernel.opt", "w") as f:
        gen_ann.write(f, gen_ann.generate([6, 5, 3], seed=1))
    formats.write_conf(str(d / "nn.conf"), type="SNN", init="kernel.opt", seed=1, train="BP",
                       sample_dir="./tests", test_dir="./tests")
    r = subprocess.run([os.path.join(BIN, "run_nn"), "-v", "-c", "nn.conf"], cwd=d, env=_env(),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ACCURACY:" in r.stdout and r.stdout.strip().endswith("/5")


def test_synthetic_rruff_records_parse(tmp_path):
    from hpnn_amd.utils import synth
    recs = synth.rruff_records(str(tmp_path), 12, seed=4)
    (tmp_path / "samples").mkdir()
    r = subprocess.run([os.path.join(BIN, "pdif"), str(tmp_path), "-i", "85", "-o", "230", "-s",
                        str(tmp_path / "samples")], capture_output=True, text=True)
    assert r.returncode == 0 and "12 samples written" in r.stdout, r.stdout + r.stderr
    for name, num in recs:
        lines = (tmp_path / "samples" / name).read_text().split("\n")
        out = lines[3].split()
        assert [i for i, v in enumerate(out) if v == "1.0"] == [num - 1]
        x = [float(v) for v in lines[1].split()]
        assert len(x) == 86 and max(x[1:]) == pytest.approx(1.0)


@pytest.mark.parametrize("tut,env", [
    ("mnist", {"NTR": "1200", "NTE": "200", "PASSES": "2", "EPOCHS": "2", "BATCH": "64"}),
    ("rruff", {"NREC": "120", "PASSES": "1", "EPOCHS": "5", "HIDDEN": "32"}),
])
def test_tutorial_end_to_end(tmp_path, tut, env):
    e = _env()
    e.update(env)
    e.update({"WORK": str(tmp_path / "run"), "FLAGS": "-c"})
    r = subprocess.run(["bash", os.path.join(ROOT, "tutorials", tut, "tutorial.sh")], cwd=tmp_path, env=e,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = (tmp_path / "run" / "raw").read_text().split("\n")
    rows = [ln.split() for ln in raw if ln.strip()]
    assert len(rows) == int(env["PASSES"])
    acc = [float(r[1]) for r in rows]
    assert all(0.0 <= a <= 100.0 for a in acc)
    assert (tmp_path / "run" / "kernel.opt").exists()


def test_monitor_renders_tutorial_raw(tmp_path):
    """ASCII monitor of a tutorial's raw file (reference: tutorial.bash:138-174 watch +
    plot.gnuplot): parses pass / accuracy / loss, skips partial lines, marks every pass"""
    from hpnn_amd.utils import monitor
    raw = tmp_path / "raw"
    raw.write_text("1 10.5 loss=2.30\n2 35.0 loss=1.90\n3 71.25\n4 \nbroken line\n")
    rows = monitor.read_raw(str(raw))
    assert rows == [(1, 10.5, 2.30), (2, 35.0, 1.90), (3, 71.25, None)]
    chart = monitor.render(rows, width=30, height=8)
    lines = chart.splitlines()
    assert lines[0].startswith("test accuracy")
    assert sum(ln.count("*") for ln in lines) == 3
    assert "pass 3: 71.25 %" in chart and "best 71.25 % at pass 3" in chart
    assert "(no data yet)" in monitor.render(monitor.read_raw(str(tmp_path / "missing")))
    r = subprocess.run([sys.executable, "-m", "hpnn_amd.utils.monitor", str(raw), "--width", "20"], cwd=ROOT,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.count("*") == 3, r.stdout + r.stderr
