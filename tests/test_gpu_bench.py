"""bench.py's output contract on the GPU, at a small configuration: one JSON
line with the metric, the roofline object (achieved / peak / frac / traffic
field) and the cpu_baseline field, after the bench's own bit-exact check of
the batch -- serial and with two batches in flight."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c2", "--steps", "3",
                        "--warmup", "1", "--no-cpu", "--copy-reps", "1", *args],
                       cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("inflight", [1, 2])
def test_bench_line_contract(inflight):
    d = _bench("--inflight", str(inflight))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["verified_bit_exact"] is True and d["errors"] == 0
    assert d["config"]["batches_in_flight"] == inflight
    assert d["config"]["frames_per_gpu"] == 262144
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["achieved"] < r["peak"]
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["algorithmic_bytes_per_launch"] == 262144 * (8 + 2 * 4096)
    assert d["cpu_baseline"] is None  # --no-cpu
