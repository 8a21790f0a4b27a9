"""bench.py's N > 1 launch on the CPU: `python bench.py --gpus N` with no
external launcher starts its N ranks itself (torch.distributed.run as a child
process) and reports an N-rank line, and a job shaped differently from --gpus
exits non-zero instead of reporting n_gpus = 1.  The
--dry-run mode runs the launch, rendezvous, shard and count all-reduce over
gloo without touching a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                          capture_output=True, text=True, timeout=240, env=env)


def _line(r):
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (r.stdout[-2000:], r.stderr[-2000:])
    return json.loads(lines[0])


def test_self_launch_two_ranks_weak():
    r = _run(["--gpus", "2", "--dry-run", "--config", "c2"], {"GEV_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r)
    assert d["n_gpus"] == 2 and d["dry_run"] is True and d["value"] is None
    c = d["decoded_per_step"]
    assert c["ranks_summed"] == 2 and c["frames"] == 2 * 262144 and c["payload_bytes"] == 2 * 262144 * 4096
    assert d["config"]["global_connections"] == 2 * d["config"]["connections_per_gpu"]


def test_self_launch_three_ranks_strong_split_covers_batch():
    import bench
    glob, _ = bench.build_layout("c5", 0, None)
    r = _run(["--gpus", "3", "--dry-run", "--config", "c5", "--scaling", "strong"], {"GEV_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r)
    assert d["n_gpus"] == 3 and d["decoded_per_step"]["ranks_summed"] == 3
    assert d["decoded_per_step"]["frames"] == glob.n_frames
    assert d["decoded_per_step"]["payload_bytes"] == glob.payload_len


def test_rccl_without_enough_devices_exits_nonzero():
    # this container has no GPU: --gpus 2 over RCCL must refuse before launching
    r = _run(["--gpus", "2", "--dry-run", "--config", "c2"], {"GEV_DIST_BACKEND": "nccl"})
    assert r.returncode != 0
    assert "needs 2 GPUs" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_world_size_mismatch_exits_nonzero():
    # launched as one rank while --gpus asks for two: no line, non-zero exit
    r = _run(["--gpus", "2", "--dry-run", "--config", "c2"],
             {"GEV_DIST_BACKEND": "gloo", "WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, drop=())
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def _fake_kfd(tmp_path, gpu_ids):
    root = tmp_path / "nodes"
    for i, g in enumerate(gpu_ids):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "gpu_id").write_text(f"{g}\n")
    return str(root)


def test_device_count_reads_kfd_topology_and_visibility(tmp_path, monkeypatch):
    import bench
    root = _fake_kfd(tmp_path, [0, 4417, 52213, 12001, 61400])  # node 0 = the CPU
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert bench.count_gpus_without_hip(root) == 4
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2")
    assert bench.count_gpus_without_hip(root) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert bench.count_gpus_without_hip(root) == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.count_gpus_without_hip(root) == 0
    assert bench.count_gpus_without_hip(str(tmp_path / "absent")) is None


# The self-launching parent with every torch device-count path booby-trapped:
# torch.cuda.device_count() (amdsmi) and torch._C._cuda_getDeviceCount() (its
# HIP fallback) raise, so any HIP-touching count in the parent ends the run.
_TRAP = r"""
import runpy, sys, torch
def _boom(*a, **k):
    raise RuntimeError("parent touched the GPU device count")
torch.cuda.device_count = _boom
torch._C._cuda_getDeviceCount = _boom
sys.argv = [sys.argv[1]] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
"""


def _run_trapped(args, env_extra):
    drop = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
    env = {k: v for k, v in os.environ.items() if k not in drop}  # (this container sets HIP_VISIBLE_DEVICES=)
    env.update(env_extra)
    return subprocess.run([sys.executable, "-c", _TRAP, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                          capture_output=True, text=True, timeout=240, env=env)


def test_parent_launches_without_hip_device_count():
    r = _run_trapped(["--gpus", "2", "--dry-run", "--config", "c2"], {"GEV_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "parent touched" not in r.stderr
    assert _line(r)["n_gpus"] == 2


def test_parent_rccl_check_uses_kfd_topology(tmp_path):
    # two GPUs in the (fake) topology: the parent's check passes without HIP and
    # launches; this container's ranks then find no device and refuse themselves
    root = _fake_kfd(tmp_path, [0, 11, 12])
    r = _run_trapped(["--gpus", "2", "--dry-run", "--config", "c2"],
                     {"GEV_DIST_BACKEND": "nccl", "GEV_KFD_TOPOLOGY": root})
    assert "parent touched" not in r.stderr
    assert "launching 2 ranks" in r.stderr
    assert r.returncode != 0 and "needs 2 GPUs" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    # one GPU in the topology: the parent refuses before launching anything
    root1 = _fake_kfd(tmp_path / "one", [0, 11])
    r = _run_trapped(["--gpus", "2", "--dry-run", "--config", "c2"],
                     {"GEV_DIST_BACKEND": "nccl", "GEV_KFD_TOPOLOGY": root1})
    assert "parent touched" not in r.stderr
    assert r.returncode == 3 and "needs 2 GPUs" in r.stderr and "launching" not in r.stderr


def _eight_rank_dry_run(config, scaling):
    import bench
    r = _run(["--gpus", "8", "--dry-run", "--config", config, "--scaling", scaling], {"GEV_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r)
    assert d["n_gpus"] == 8 and d["dry_run"] is True and d["value"] is None and d["scaling"] == scaling
    c = d["decoded_per_step"]
    assert c["ranks_summed"] == 8 and c["errors"] == 0
    # every rank's batch fits one MI355X with room to spare (checked again on the device, bench.main)
    assert 0 < d["hbm_need_bytes_per_rank"] < 0.9 * bench.HBM_BYTES_PER_GPU
    return d, c


@pytest.mark.parametrize("config,frames,size", [("c2", 262144, 4096), ("c3", 1048576, 65536)])
def test_eight_ranks_weak_counts_every_rank(config, frames, size):
    """The driver's top scaling point: 8 self-launched
    ranks over gloo, weak scaling of C2 and of the headline C3 (the driver's
    default) -- one JSON line, n_gpus 8, the count all-reduce summing 8 ranks'
    full batches."""
    d, c = _eight_rank_dry_run(config, "weak")
    assert c["frames"] == 8 * frames and c["payload_bytes"] == 8 * frames * size
    assert d["config"]["global_connections"] == 8 * d["config"]["connections_per_gpu"]


def test_eight_ranks_strong_c4_split_covers_batch():
    """8 ranks, C4 strong scaling: the LPT shares of the one global batch sum
    to exactly its frames and payload bytes."""
    import bench
    glob, _ = bench.build_layout("c4", 0, None)
    d, c = _eight_rank_dry_run("c4", "strong")
    assert c["frames"] == glob.n_frames and c["payload_bytes"] == glob.payload_len
    assert d["config"]["global_connections"] == glob.n_conns


def test_hbm_need_of_the_headline_batch_fits_one_gpu():
    """C3 at full size (64 GiB in, 64 GiB out) is checked up front against the
    device's free memory; the estimate itself fits an MI355X's 288 GB, and a
    second batch in flight adds its outputs and scratch."""
    import bench
    lay, _ = bench.build_layout("c3", 0, None)
    one, two = bench.hbm_need_bytes(lay, 1), bench.hbm_need_bytes(lay, 2)
    assert 2 * lay.payload_len < one < bench.HBM_BYTES_PER_GPU
    assert two - one >= lay.payload_padded
