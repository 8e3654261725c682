"""bench.py honours the driver's contract for every model it offers: one JSON line with the
required keys, the timed step count, and the config's batch / scaling."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


@pytest.mark.parametrize("model,batch,scaling", [("mnist", 65536, "weak"), ("rruff", 16384, "weak"),
                                                 ("synth", 8192, "strong")])
def test_bench_contract(gpu, model, batch, scaling):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                            "HPNN_DP_FORCE", "HPNN_BENCH_REHEARSE")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", model, "--steps", "3", "--warmup",
                        "1", "--graph-steps", "2"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert KEYS <= set(d), KEYS - set(d)
    assert d["steps"] == 3 and d["warmup"] == 1 and d["n_gpus"] == 1 and d["dtype"] == "bf16"
    assert d["scaling"] == scaling and d["config"]["global_batch"] == batch and d["higher_is_better"] is True
    assert d["value"] > 0 and abs(d["value"] - batch / (d["ms_per_step"] / 1e3)) <= 1e-6 * d["value"]
    assert d["config"]["hip_graph"] is True
