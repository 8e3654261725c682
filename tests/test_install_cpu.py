"""`make install PREFIX=...` and a third-party C program built against the installed
library through its pkg-config file (the reference installs libhpnn.la, libhpnn.h,
libhpnn/*.h and libhpnn.pc: src/Makefile.am:12-41, src/libhpnn.pc.in).

The program is plain C: it trains the 4-8-4 ANN regression config (BASELINE.json's CPU
plumbing config) on the CPU engine and writes kernel.opt.  pkg-config itself is used when
it is installed; otherwise the .pc file is expanded here with pkg-config's own rules
(${var} substitution, Cflags / Libs fields)."""
import os
import re
import shutil
import subprocess

import numpy as np

from hpnn_amd.utils import formats

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROGRAM = r"""
#include <stdio.h>
#include <libhpnn.h>

int main(int argc, char **argv) {
    nn_def *conf;
    FILE *fp;
    if (argc < 2) return 2;
    nn_init_all(0);
    conf = nn_load_conf(argv[1]);
    if (conf == NULL) return 3;
    if (nn_get_n_inputs(conf) != 4 || nn_get_n_outputs(conf) != 4 || nn_get_h_neurons(conf, 0) != 8) return 4;
    if (!nn_train_kernel(conf)) return 5;
    fp = fopen("kernel.opt", "w");
    if (fp == NULL) return 6;
    nn_dump_kernel(conf, fp);
    fclose(fp);
    printf("trained %s with %s\n", nn_return_name(conf), nn_return_version());
    nn_deinit_conf(conf);
    nn_deinit_all();
    return 0;
}
"""


def _pkg_config(pc_dir, *args):
    if shutil.which("pkg-config"):
        env = dict(os.environ, PKG_CONFIG_PATH=pc_dir)
        return subprocess.run(["pkg-config", *args, "libhpnn"], env=env, capture_output=True, text=True,
                              check=True).stdout.split()
    # pkg-config semantics for the fields used here: "name=value" variables expanded
    # recursively with ${name}, then the requested fields
    vars_, fields = {}, {}
    for line in open(os.path.join(pc_dir, "libhpnn.pc")):
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        m = re.match(r"^([A-Za-z_][\w.]*)\s*=\s*(.*)$", line)
        if m:
            vars_[m.group(1)] = m.group(2)
            continue
        m = re.match(r"^([A-Za-z.]+):\s*(.*)$", line)
        if m:
            fields[m.group(1)] = m.group(2)

    def expand(v):
        for _ in range(10):
            v = re.sub(r"\$\{(\w+)\}", lambda mm: vars_[mm.group(1)], v)
        return v
    out = []
    if "--cflags" in args:
        out += expand(fields.get("Cflags", "")).split()
    if "--libs" in args:
        out += expand(fields.get("Libs", "")).split()
    return out


def test_install_and_link_with_pkg_config(tmp_path):
    prefix = str(tmp_path / "prefix")
    r = subprocess.run(["make", "-C", ROOT, "install", f"PREFIX={prefix}"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    for f in ("lib/libhpnn.so", "include/libhpnn.h", "include/libhpnn/common.h", "include/libhpnn/ann.h",
              "lib/pkgconfig/libhpnn.pc", "bin/train_nn", "bin/run_nn"):
        assert os.path.exists(os.path.join(prefix, f)), f
    pc = os.path.join(prefix, "lib", "pkgconfig")
    flags = _pkg_config(pc, "--cflags", "--libs")
    assert f"-I{prefix}/include" in flags and "-lhpnn" in flags
    work = tmp_path / "work"
    (work / "samples").mkdir(parents=True)
    src = work / "prog.c"
    src.write_text(PROGRAM)
    exe = str(work / "prog")
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", str(src), "-o", exe, *flags], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    # 4-8-4 ANN regression on the CPU engine (HPNN_FORCE_CPU=1), 8 samples
    rng = np.random.default_rng(3)
    for i in range(8):
        x = rng.uniform(-1, 1, 4)
        t = np.full(4, -1.0)
        t[int(np.argmax(x))] = 1.0
        formats.write_sample(str(work / "samples" / f"s{i:03d}.txt"), x, t)
    formats.write_conf(str(work / "nn.conf"), name="install", type="ANN", seed=10958, inputs=4, hiddens=[8],
                       outputs=4, train="BP", sample_dir="./samples", test_dir="./samples")
    env = dict(os.environ, HPNN_FORCE_CPU="1")
    env.pop("LD_LIBRARY_PATH", None)  # the rpath from the .pc Libs must be enough
    r = subprocess.run([exe, "nn.conf"], cwd=str(work), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "trained install" in r.stdout
    k = formats.read_kernel(str(work / "kernel.opt"))
    assert [w.shape for w in k["weights"]] == [(8, 4), (4, 8)]
    # the installed CLI runs against the installed library too
    r = subprocess.run([os.path.join(prefix, "bin", "run_nn"), "nn.conf"], cwd=str(work), env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
