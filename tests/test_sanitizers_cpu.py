"""Host-code sanitizers (Race detection / sanitizers): the C API, runtime, CPU
engine, sample/state I/O and CLIs built with AddressSanitizer + UBSan (`make asan`,
build/asan/*) run the CPU workflows -- online and batched training, exact resume, pack
files, evaluation -- with leak detection on; any sanitizer report fails the test.
(GPU-side sanitizers are not available on this pool; device code is covered by the
bitwise-determinism checks of tests/test_model_gpu.py.)"""
import os
import shutil
import subprocess

import pytest

from tests.test_aux_cpu import _conf, _dataset

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "build", "asan")


@pytest.fixture(scope="module")
def asan_bins():
    if shutil.which("make") is None or shutil.which(os.environ.get("CXX", "g++")) is None:
        pytest.skip("no host toolchain")
    r = subprocess.run(["make", "-C", ROOT, "-j8", "asan"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return ASAN


def _san(cmd, cwd):
    env = dict(os.environ, HPNN_FORCE_CPU="1", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=600)
    log = r.stdout + r.stderr
    assert "AddressSanitizer" not in log and "LeakSanitizer" not in log and "runtime error:" not in log, log[-4000:]
    assert r.returncode == 0, log[-4000:]
    return r.stdout


def test_cli_workflows_clean_under_asan_ubsan(asan_bins, tmp_path):
    d = str(tmp_path)
    _dataset(os.path.join(d, "samples"))
    _conf(d)
    tn, rn, pk = (os.path.join(asan_bins, x) for x in ("train_nn", "run_nn", "pack_nn"))
    _san([tn, "-vv", "nn.conf"], d)                                   # online BPM (reference loop)
    _san([tn, "-vv", "-b", "5", "-e", "2", "-r", "st.bin", "nn.conf"], d)  # batched, writes state
    out = _san([tn, "-vv", "-b", "5", "-e", "1", "-r", "st.bin", "nn.conf"], d)  # resumes
    assert "momentum restored" in out
    _san([pk, "samples", "p.hpnb"], d)
    _conf(d, samples="./p.hpnb")
    _san([tn, "-T", "-b", "7", "-M", "m.jsonl", "nn.conf"], d)
    out = _san([rn, "-vv", "nn.conf"], d)
    assert out.count("TESTING FILE") == 24
