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


def _bench_2rank(config, port, steps=3):
    """The driver's N > 1 launch (torch.distributed.run, one process per rank)
    with 2 ranks sharing this one GPU over gloo (RCCL allows one rank per
    device): per-rank batches, bit-exact verification on every rank, the count
    all-reduce, max-over-ranks timing and the rank-0-only JSON line."""
    env = dict(os.environ, GEV_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--config", config, "--steps", str(steps), "--warmup", "1", "--no-cpu",
                        "--copy-reps", "0"], cwd=ROOT, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    return json.loads(lines[0])


def test_bench_two_ranks_weak_c2():
    d = _bench_2rank("c2", 29611)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["errors"] == 0
    c = d["decoded_per_step"]
    assert c["ranks_summed"] == 2 and c["frames"] == 2 * 262144 and c["payload_bytes"] == 2 * 262144 * 4096
    assert d["config"]["global_connections"] == 2 * d["config"]["connections_per_gpu"]


def test_bench_self_launch_two_ranks_gloo():
    """`bench.py --gpus 2` with no launcher starts its own two ranks (here both
    on this GPU over gloo) and reports n_gpus 2, not a one-GPU line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["GEV_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "c2",
                        "--steps", "2", "--warmup", "1", "--no-cpu", "--copy-reps", "0"],
                       cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["decoded_per_step"]["ranks_summed"] == 2 and d["value"] > 0


def test_bench_rccl_more_ranks_than_gpus_exits_nonzero():
    import torch
    n = torch.cuda.device_count() + 1
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GEV_DIST_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--config", "c2",
                        "--steps", "1", "--warmup", "0", "--no-cpu", "--copy-reps", "0"],
                       cwd=ROOT, capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert f"needs {n} GPUs" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_two_ranks_strong_c4():
    import bench
    glob, _ = bench.build_layout("c4", 0, None)
    d = _bench_2rank("c4", 29612, steps=2)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["errors"] == 0
    c = d["decoded_per_step"]
    # the two LPT shares together are exactly the global batch
    assert c["frames"] == glob.n_frames and c["payload_bytes"] == glob.payload_len
    assert d["config"]["global_connections"] == glob.n_conns
