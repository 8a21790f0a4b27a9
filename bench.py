#!/usr/bin/env python3
"""bench.py -- device-resident WebSocket frame decode + payload unmask on MI355X.

Metric (BASELINE.json): "GiB/s WS payload unmasked (device-resident) +
frames/s, 64 KiB masked frames".  One step = one pass of the hot path
(gevws_decode_batch_async: header walk, scan, record emit, unmask/compact)
over one synthetic batch already resident in HBM, plus the RCCL all-reduce of
the decoded {frames, payload bytes, errors} counts when N > 1.

Default workload (N=1): C3 = 1 048 576 masked binary 64 KiB frames (h = 14)
over 16 384 connections, generated on the device (seeded splitmix64).  With
N > 1 every rank decodes its own connections' batch of the same size (weak
scaling: connections shard by GPU, the payload never crosses GPUs).

Prints ONE JSON line (rank 0).  `roofline` is the unmask kernel's algorithmic
bytes (h + 2L per frame) over its mean HIP-event duration in the
timed region; `cpu_baseline` is the C restatement of the reference per-frame
UnPacket pipeline (oracle/ws_ref.c) timed on this host's cores on a bounded
sample of the same workload.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`python bench.py --gpus N` (N > 1) without a launcher starts its N ranks itself
(torch.distributed.run as a child process, before anything touches a GPU) and
exits with their status; a rank whose WORLD_SIZE differs from --gpus, or an
RCCL job with fewer GPUs than ranks, exits non-zero without a line.
`--dry-run` runs only the launch / shard / count-reduce plumbing (gloo, no GPU).

Measurement options (not the contract line's defaults): --inflight M (M
batches in flight on M streams), --emulate-shard R/N (rank R's LPT share of an
N-way strong split, on one GPU), --walk-variant / --unmask-variant /
--split-lanes (A/B).
The split header walk's auto choice (GEVWS_TUNE_SPLIT_LANES 0) looks at the
previous finished decode on the context: the untimed verify decode walks
unsplit, the warmup and timed steps split when that decode showed long chains
of small frames on few connections (C4's 8-way share).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "GiB/s WS payload unmasked (device-resident) + frames/s, 64 KiB masked frames"


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def build_layout(name: str, rank: int, conns: int | None, world: int = 1, scaling: str = "weak"):
    """Weak: every rank its own batch of the config's shape (per-rank seed).
    Strong: one global batch (same seed on every rank), connections assigned to
    ranks by greedy LPT over stream bytes; this rank decodes its share."""
    from gev_amd import workloads as w
    from gev_amd.dist import rank_seed
    if scaling == "strong":
        glob, _ = build_layout(name, 0, conns)
        return w.shard_lpt(glob, rank, world), glob
    seed = rank_seed(0x67657600, rank)
    if name == "c1":  # device-resident batch of the C1 plumbing config's frames (128 B masked text)
        lay = w.uniform(conns or 65536, 16, 128, opcode=0x1, seed=seed,
                        name="C1-shaped: 1048576 x 128 B masked text frames")
    elif name == "c3":
        lay = w.config_c3(seed=seed, n_conns=conns or 16384)
    elif name == "c2":
        lay = w.config_c2(seed=seed, n_conns=conns or 4096)
    elif name == "c4":
        lay = w.config_c4(total_payload=16 << 30, n_conns=conns or 65536, seed=seed)
    elif name == "c5":
        lay = w.config_c5(n_conns=conns or 256, seed=seed)
    else:
        raise SystemExit(f"unknown config {name}")
    return lay, lay


HBM_BYTES_PER_GPU = 288 * 10**9  # MI355X HBM3E


def hbm_need_bytes(lay, inflight: int = 1) -> int:
    """Device memory one rank allocates for its batch, an upper estimate
    checked before anything is allocated: the input arena (+ pad), the frame
    descriptors and connection table, and per batch in flight the outputs
    (payload arena, 32-byte records, 24-byte per-connection results) and the
    decode context's scratch -- the walk's 8-byte frame entries (one per 64
    input bytes, in 32-entry slot runs per connection), the output-tile map
    and the block partials (gevws_walk.hip decode_front)."""
    entries = 32 * ((lay.arena_bytes >> 11) + lay.n_conns + 1) * 8
    scratch = entries + (lay.payload_padded // 4096 + 2) * 4 + lay.n_conns * 64 + (1 << 20)
    out = lay.payload_padded + 16 + lay.n_frames * 32 + lay.n_conns * 24 + 4096
    return lay.arena_bytes + 64 + lay.desc.nbytes + lay.conns.nbytes + inflight * (out + scratch)


def cpu_sample_layout(name: str, mib: int = 256):
    """A bounded sample of the same workload for the CPU baseline: `mib` MiB of
    payload (>= 64 MiB of input per thread, so the sample is not cache-resident)."""
    from gev_amd import workloads as w
    if name == "c3":
        n = mib * 16
        return w.uniform(16 * mib // 256, 256, 65536, seed=1,
                         name=f"{n} x 64 KiB masked binary frames ({mib} MiB payload)")
    if name == "c2":
        n = mib * 256
        return w.uniform(64 * mib // 256, 1024, 4096, seed=1,
                         name=f"{n} x 4 KiB masked binary frames ({mib} MiB payload)")
    if name == "c4":
        return w.config_c4(total_payload=mib << 20, n_conns=4 * mib, seed=1)
    if name == "c1":
        n = mib * 8192
        return w.uniform(n // 16, 16, 128, opcode=0x1, seed=1, name=f"{n} x 128 B masked text frames ({mib} MiB payload)")
    return w.config_c5(n_conns=mib // 8, seed=1)


def host_cpu_info() -> dict:
    """The host the CPU baseline runs on: model, logical CPUs (nproc), the CPUs
    this process may run on (affinity) and the cgroup CPU quota, if any."""
    info = {"model": None, "nproc": os.cpu_count(), "affinity": None, "cgroup_cpu_quota": None}
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                info["model"] = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return info


def all_host_threads() -> int:
    """One thread per CPU this process may use (nproc unless an affinity mask
    narrows it) -- SURVEY.md §8d's "all host cores"."""
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_baseline(name: str, seconds: float, threads: int, vectorized: bool = False, alloc: str = "fresh"):
    import numpy as np
    from gev_amd import workloads as w
    from oracle import ref
    # 64 MiB of payload per thread up to 4 GiB in all (>= 16 MiB per thread at
    # 256 threads), at least 256 MiB: never cache-resident
    lay = cpu_sample_layout(name, min(4096, max(256, 64 * threads)))
    arena = np.concatenate([w.synth_host(lay), np.zeros(64, np.uint8)])
    secs, pb, nf = ref.bench_pipeline(arena, lay.conns[:, 0], lay.conns[:, 1], threads=threads,
                                      min_seconds=seconds, vectorized=vectorized, alloc=alloc)
    where = (f"make() from a per-thread bump arena of {ref.fresh_arena_bytes() >> 20} MiB (2 x the LLC a CPU sees, "
             "at least 64 MiB; fresh memory as Go's swept spans)" if alloc == "fresh" else
             "make() as calloc/free per frame (glibc recycles one cache-warm chunk)")
    return dict(value=round(pb / secs / 2**30, 4), unit="GiB/s", cores=threads, kind="port", alloc=alloc,
                frames_per_s=round(nf / secs, 1), host=host_cpu_info(),
                sample=(f"{lay.name}, {lay.n_conns} connections round-robin over {threads} thread(s), "
                        f"repeated for >= {seconds:.0f} s; oracle/ws_ref.c per-frame UnPacket pipeline "
                        f"(header parse, zero-filled make, ring Read copy, Cipher u64 loop); {where}; "
                        + ("gcc -O3 -mavx2 (auto-vectorised)" if vectorized else "gcc -O2 -fno-tree-vectorize")))


def load_traffic(config_name: str):
    """HBM bytes per unmask launch from a committed rocprofv3 --pmc pass (see
    profiles/README.md) and where they come from (file and
    commit), or (None, None).  The passes are taken at N = 1, so the figure
    applies to a rank's launch only when that rank runs the same batch (N = 1,
    or weak scaling)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None, None
    try:
        d = json.load(open(p))
        e = d.get(config_name)
        if e is None:
            return None, None
        return int(e["hbm_bytes_per_launch"]), {"file": e.get("source"), "commit": e.get("commit"),
                                                "kernel": e.get("kernel")}
    except Exception:
        return None, None


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _env_device_list(name: str):
    """Entries of a *_VISIBLE_DEVICES variable (None when unset)."""
    v = os.environ.get(name)
    if v is None:
        return None
    return [x for x in v.split(",") if x.strip()]


def count_gpus_without_hip(kfd_root: str | None = None):
    """GPUs this job may use, counted WITHOUT any HIP call (the self-launching
    parent must not hold a HIP runtime while its ranks run): the KFD topology
    nodes with a non-zero gpu_id (CPU nodes have 0), narrowed by
    ROCR_VISIBLE_DEVICES and then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES.
    None when the topology is not readable -- the caller then skips its check
    and leaves the refusal to each rank's check_world.  (GEV_KFD_TOPOLOGY
    points the CPU tests at a fake topology.)"""
    if kfd_root is None:
        kfd_root = os.environ.get("GEV_KFD_TOPOLOGY", "/sys/class/kfd/kfd/topology/nodes")
    try:
        nodes = os.listdir(kfd_root)
    except OSError:
        return None
    n = 0
    for node in nodes:
        try:
            with open(os.path.join(kfd_root, node, "gpu_id")) as f:
                n += int(f.read().strip() or 0) != 0
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        lst = _env_device_list(var)
        if lst is not None:
            n = min(n, len(lst))
    return n


def launch_ranks(n: int, argv: list) -> int:
    """`bench.py --gpus N` run without a launcher: start the N rank processes
    itself -- torch.distributed.run as a CHILD process (never an exec), one rank
    per GPU, rendezvous on 127.0.0.1 -- and return its exit status.  Rank 0's
    JSON line reaches stdout through the inherited descriptor.  Nothing here
    touches the GPU: the device count comes from the KFD topology in sysfs
    (count_gpus_without_hip), never from torch.cuda (whose device_count()
    falls back to a HIP call when amdsmi fails), so the ranks are the only
    processes that open a device.  Without a readable topology the check is
    left to the ranks (check_world)."""
    import subprocess
    if _backend() == "nccl":
        ndev = count_gpus_without_hip()
        if ndev is not None and ndev < n:
            log(f"error: --gpus {n} needs {n} GPUs for RCCL (one rank per device); {ndev} visible")
            return 3
        if ndev is None:
            log("device count unavailable without HIP (no KFD topology); each rank checks its own")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    log(f"launching {n} ranks: {' '.join(cmd[1:7])} ...")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def _backend() -> str:
    return os.environ.get("GEV_DIST_BACKEND", "nccl")


def _visible_devices() -> int:
    """Inside a rank only (a rank opens its GPU anyway): torch's count."""
    import torch
    return torch.cuda.device_count()


def check_world(args, world: int, need_devices: bool) -> None:
    """Refuse to print a line for a job shaped differently from what was asked:
    WORLD_SIZE must be --gpus, and under RCCL every rank needs its own device
    (checked in the rank, also for --dry-run: a dry run over RCCL is refused
    the same way)."""
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to report "
                         f"n_gpus={world} for a {args.gpus}-GPU run")
    if need_devices and _backend() == "nccl" and world > 1 and _visible_devices() < world:
        raise SystemExit(f"bench: {world} ranks over RCCL needs {world} GPUs (one per rank); "
                         f"{_visible_devices()} visible")


def dry_run(args) -> None:
    """--dry-run: the N > 1 plumbing without a GPU (a CPU test of the launch):
    rendezvous, this rank's share of the batch, the count all-reduce and the
    max-over-ranks time, over gloo.  Counts come from the layouts, nothing is
    decoded or timed, and `value` is null: not a measurement."""
    import torch
    from gev_amd import dist
    world, rank, _ = dist.env()
    check_world(args, world, need_devices=True)
    if world > 1 and dist.backend() != "gloo":
        raise SystemExit("bench --dry-run: GEV_DIST_BACKEND=gloo (no GPU is used)")
    dist.init(dist.backend(), None)
    scaling = args.scaling or ("strong" if args.config == "c4" else "weak")
    lay, glob = build_layout(args.config, rank, args.conns, world, scaling)
    counts = torch.tensor([lay.n_frames, lay.payload_len, 0], dtype=torch.int64)
    dist.reduce_counts(counts)
    need_max = int(dist.max_over_ranks(float(hbm_need_bytes(lay, max(1, args.inflight))), "cpu"))
    dist.barrier()
    elapsed = dist.max_over_ranks(0.0, "cpu")
    if rank == 0:
        c = counts.tolist()
        print(json.dumps({
            "metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "steps": 0,
            "warmup": 0, "ms_per_step": None, "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "dtype": "u8", "data": "dry run: layouts only, nothing decoded",
            "config": {"workload": lay.name, "connections_per_gpu": lay.n_conns,
                       "global_connections": glob.n_conns if scaling == "strong" else glob.n_conns * world,
                       "parallelism": f"connections sharded over {world} rank(s); {dist.backend()} all-reduce of counts"},
            "decoded_per_step": {"frames": c[0], "payload_bytes": c[1], "errors": c[2], "ranks_summed": world},
            "hbm_need_bytes_per_rank": need_max, "max_over_ranks_s": elapsed, "dry_run": True}), flush=True)
    dist.finalize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=["c1", "c2", "c3", "c4", "c5"])
    ap.add_argument("--conns", type=int, default=None)
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None,
                    help="weak: each GPU its own batch of the config's shape (default for c2/c3/c5); "
                         "strong: one global batch sharded over the GPUs by LPT (default for c4)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads-multi", type=int, default=0,
                    help="threads of the all-cores CPU baseline (0 = every CPU this process may use)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--copy-reps", type=int, default=5, help="streaming-copy ceiling reps (0 = skip)")
    ap.add_argument("--copy-interleave", type=int, default=0,
                    help="R rounds of [decode, size-matched aligned copy] after the timed region: the unmask "
                         "against the copy rate in the same clock state (0 = skip)")
    ap.add_argument("--walk-variant", type=int, default=None, help="A/B: header walk variant (GEVWS_TUNE_WALK_VARIANT)")
    ap.add_argument("--unmask-variant", type=int, default=None, help="A/B: unmask kernel variant")
    ap.add_argument("--unmask-grid", type=int, default=None,
                    help="A/B: cap the unmask's workgroups (GEVWS_TUNE_UNMASK_GRID; leaves CU slots for a batch in flight)")
    ap.add_argument("--split-lanes", type=int, default=None,
                    help="A/B: split header walk lanes per connection (GEVWS_TUNE_SPLIT_LANES; 0 = auto, 1 = off)")
    ap.add_argument("--emulate-shard", default=None, metavar="R/N",
                    help="projection, not the contract line: decode only rank R's LPT share of an N-way strong "
                         "split of the global batch, on this one GPU")
    ap.add_argument("--inflight", type=int, default=1,
                    help="batches in flight: M contexts on M streams with M output arenas, step i on slot i %% M "
                         "(a server loop: one batch's header walk overlaps the previous batch's unmask)")
    ap.add_argument("--input-mem", choices=["default", "fine", "uncached"], default="default",
                    help="measurement: the input arena's memory kind (gevws_device_alloc)")
    ap.add_argument("--dry-run", action="store_true",
                    help="N > 1 plumbing only, no GPU (launch, shard, count all-reduce over gloo); value is null")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.dry_run:
        return dry_run(args)

    import numpy as np
    import torch

    import gev_amd
    from gev_amd import dist
    from gev_amd.workloads import size_histogram

    world, rank, local = dist.env()
    check_world(args, world, need_devices=True)
    gpu = local % max(torch.cuda.device_count(), 1)  # == local on a node with one rank per GPU
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist.init(dist.backend(), dev)  # RCCL over xGMI when WORLD_SIZE > 1

    from gev_amd import _abi
    M = max(1, args.inflight)
    engs = [gev_amd.Engine(gpu) for _ in range(M)]  # one context (scratch) per stream
    eng = engs[0]
    for e in engs:
        if args.walk_variant is not None:
            e.set_tuning(_abi.TUNE_WALK_VARIANT, args.walk_variant)
        if args.unmask_variant is not None:
            e.set_tuning(_abi.TUNE_UNMASK_VARIANT, args.unmask_variant)
        if args.split_lanes is not None:
            e.set_tuning(_abi.TUNE_SPLIT_LANES, args.split_lanes)
        if args.unmask_grid is not None:
            e.set_tuning(_abi.TUNE_UNMASK_GRID, args.unmask_grid)
    t_setup = time.time()
    scaling = args.scaling or ("strong" if args.config == "c4" else "weak")
    emulated = None
    if args.emulate_shard:
        er, en = (int(x) for x in args.emulate_shard.split("/"))
        if world != 1 or not 0 <= er < en:
            raise SystemExit("--emulate-shard R/N: one process, 0 <= R < N")
        scaling, emulated = "strong", {"rank": er, "world": en}
        lay, glob = build_layout(args.config, er, args.conns, en, "strong")
    else:
        lay, glob = build_layout(args.config, rank, args.conns, world, scaling)
    if lay.n_frames == 0:
        raise SystemExit(f"rank {rank}: no connections in this rank's share ({glob.n_conns} in the batch)")
    log(f"rank {rank}: {lay.name}: {lay.n_frames} frames, {lay.n_conns} connections, "
        f"{lay.arena_bytes / 2**30:.2f} GiB in, {lay.payload_padded / 2**30:.2f} GiB out")
    # every rank checks its device memory before allocating: a rank that cannot
    # hold its batch exits non-zero here (no line, nothing launched)
    need = hbm_need_bytes(lay, M)
    free_b, total_b = torch.cuda.mem_get_info(dev)
    if need > free_b:
        raise SystemExit(f"rank {rank}: the batch needs {need / 2**30:.1f} GiB of device memory, "
                         f"{free_b / 2**30:.1f} GiB free of {total_b / 2**30:.1f} GiB; refusing to run")
    if args.input_mem == "default":
        arena = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
        arena[lay.arena_bytes:] = 0
    else:  # measurement: the input arena in fine-grained / uncached device memory (zeroed)
        arena = gev_amd.DeviceArena(gpu, lay.arena_bytes + gev_amd.IN_PAD,
                                    gev_amd.MEM_FINE if args.input_mem == "fine" else gev_amd.MEM_UNCACHED)
    desc = torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev)
    conns = torch.from_numpy(lay.conns.copy()).to(dev)
    eng.synth(arena, desc, lay.n_frames, lay.seed)
    max_frames, cap = lay.n_frames, lay.payload_padded
    out = eng.alloc_batch(lay.n_conns, max_frames, cap)

    # correctness gate (outside the timed region): decode(mask(P)) == P on every byte
    eng.decode_async(arena, lay.arena_bytes, conns, lay.n_conns, out, max_frames, cap)
    mism = torch.zeros(1, dtype=torch.int64, device=dev)
    eng.verify(desc, lay.n_frames, lay.seed, out, mism)
    torch.cuda.synchronize()
    s = out.summary_host()
    mismatch = int(mism.item())
    if mismatch or int(s["frames"]) != lay.n_frames or int(s["payload_len"]) != lay.payload_len:
        raise SystemExit(f"verification failed: mismatch={mismatch} frames={int(s['frames'])}")
    log(f"rank {rank}: setup+verify {time.time() - t_setup:.1f}s, bit-exact")

    counts = torch.zeros(3, dtype=torch.int64, device=dev)
    sel = torch.tensor([0, 2, 3], dtype=torch.int64, device=dev)
    sum64 = out.summary.view(torch.int64)
    outs = [out] + [e.alloc_batch(lay.n_conns, max_frames, cap) for e in engs[1:]]
    # (alternate priorities: each priority level has its own hardware queues,
    # while same-priority streams share their level's 3 -- tools/queue_probe.hip
    # -- and two of torch's pool streams landed on one here, which serialised
    # the batches in flight)
    streams = [None] if M == 1 else [torch.cuda.Stream(dev, priority=-(k % 2)) for k in range(M)]
    main_stream = torch.cuda.current_stream()
    n_step = [0]

    def step():
        k = n_step[0] % M
        n_step[0] += 1
        engs[k].decode_async(arena, lay.arena_bytes, conns, lay.n_conns, outs[k], max_frames, cap,
                             stream=streams[k])
        if world > 1:  # decoded {frames, payload bytes, errors}, summed over GPUs (N = 1: read after the loop)
            if M > 1:
                engs[k].order_after_last(main_stream)
            torch.index_select(outs[k].summary.view(torch.int64), 0, sel, out=counts)
            dist.reduce_counts(counts)

    for _ in range(args.warmup):
        step()
    for e in engs:
        e.timing()  # drop anything recorded so far
    dist.barrier()
    torch.cuda.synchronize()
    for e in engs:
        e.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    phases, calls = [0.0] * 4, 0
    for e in engs:
        e.set_timing(False)
        ph, cl = e.timing()
        phases = [a + b for a, b in zip(phases, ph)]
        calls += cl
    elapsed = dist.max_over_ranks(t1 - t0, dev)
    # the timed steps' own output checked too (outside the timed region): every
    # slot's last batch, decode(mask(P)) == P on every byte
    for k in range(M):
        mism.zero_()
        engs[k].verify(desc, lay.n_frames, lay.seed, outs[k], mism)
        torch.cuda.synchronize()
        sk = outs[k].summary_host()
        if int(mism.item()) or int(sk["status"]) != 0 or int(sk["frames"]) != lay.n_frames:
            raise SystemExit(f"verification of the timed output failed (slot {k}): mismatch={int(mism.item())} "
                             f"status={int(sk['status'])}")
    del desc

    last = engs[(args.steps + args.warmup - 1) % M]  # the context of the last step
    walk_info = {"split_lanes": last.last_split_lanes, "split_fallbacks": last.last_split_fallbacks}
    # achievable-bandwidth ceiling on this box, after the timed region: the
    # unmask kernel's streaming loop minus XOR / frame lookup (gevws_copy_async)
    # over the same byte count into the payload arena -- from the payload's
    # unaligned source offset (the first payload byte) and from an aligned one
    # (offset 0: a float4 copy, the chip's copy rate), each with non-temporal
    # loads (as the unmask's streaming path) and with plain loads; the fastest
    # of the four is the ceiling
    copy_gbps = None
    copy_by_load = {}
    if args.copy_reps > 0:
        from gev_amd.workloads import header_len
        src_off = int(header_len(lay.desc["length"][:1], lay.desc["masked"][:1], lay.desc["len_form"][:1])[0])
        n_copy = min(lay.payload_padded, lay.arena_bytes - src_off) // 16 * 16
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        span = 0x20000000 | (4 * ncu)  # the unmask's layout: wave-contiguous 16 KiB spans, 4 workgroups per CU
        for name, flag, so in (("nt", 0, src_off), ("plain", 0x40000000, src_off),
                               ("nt_aligned", 0, 0), ("plain_aligned", 0x40000000, 0),
                               ("nt_aligned_wavespan", span, 0), ("plain_aligned_wavespan", span | 0x40000000, 0)):
            eng.copy_(out.payload, arena, n_copy, src_offset=so, grid=flag)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.copy_reps):
                eng.copy_(out.payload, arena, n_copy, src_offset=so, grid=flag)
            e1.record()
            torch.cuda.synchronize()
            copy_by_load[name] = round(2 * n_copy / (e0.elapsed_time(e1) / args.copy_reps / 1e3) / 1e9, 1)
        copy_gbps = max(copy_by_load.values())
    # --copy-interleave R: R rounds of [one decode (its unmask timed by HIP
    # events), one aligned copy of the same byte count (plain and
    # non-temporal loads, the faster)] back to back, so the ceiling is taken in
    # the same clock / thermal state as the unmask it is compared with
    interleaved = None
    if args.copy_interleave > 0:
        n_copy = min(lay.payload_padded, lay.arena_bytes) // 16 * 16
        ums, cms = [], []
        for _ in range(args.copy_interleave):
            engs[0].set_timing(True)
            engs[0].decode_async(arena, lay.arena_bytes, conns, lay.n_conns, outs[0], max_frames, cap,
                                 stream=streams[0])
            engs[0].set_timing(False)
            engs[0].order_after_last(torch.cuda.current_stream())
            best = None
            for flag in (0, 0x40000000):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                eng.copy_(out.payload, arena, n_copy, src_offset=0, grid=flag)
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1)
                best = t if best is None else min(best, t)
            ph, cl = engs[0].timing()
            ums.append(ph[3] / max(cl, 1))
            cms.append(best)
        um, cm = sorted(ums)[len(ums) // 2], sorted(cms)[len(cms) // 2]
        ua = lay.algorithmic_bytes() / (um / 1e3) / 1e9
        cg = 2 * n_copy / (cm / 1e3) / 1e9
        interleaved = {"rounds": args.copy_interleave, "unmask_ms": round(um, 4), "copy_ms": round(cm, 4),
                       "unmask_GBps": round(ua, 1), "copy_GBps": round(cg, 1), "frac_of_copy": round(ua / cg, 4)}
    if world == 1:
        torch.index_select(sum64, 0, sel, out=counts)
    c = counts.cpu().numpy()
    frames_step, payload_step, errors = int(c[0]), int(c[1]), int(c[2])
    ms_step = elapsed / args.steps * 1e3
    value = payload_step * args.steps / elapsed / 2**30
    mean_ms = [p / max(calls, 1) for p in phases]
    unmask_ms = mean_ms[3]
    alg_bytes = lay.algorithmic_bytes()
    achieved = alg_bytes / (unmask_ms / 1e3) / 1e9
    pipeline_gbps = alg_bytes / (sum(mean_ms) / 1e3) / 1e9

    if rank != 0:
        dist.finalize()
        return
    # (the committed counts describe the default kernels on the full batch)
    traffic, traffic_src = (load_traffic(args.config)
                            if (scaling == "weak" or world == 1) and not emulated and not args.unmask_variant
                            and not args.walk_variant and not args.unmask_grid else (None, None))
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: masked frames generated on the device (seeded splitmix64 payloads and keys)",
        "config": {"workload": lay.name, "connections_per_gpu": lay.n_conns, "frames_per_gpu": lay.n_frames,
                   "payload_bytes_per_gpu": lay.payload_len, "input_bytes_per_gpu": lay.arena_bytes,
                   "global_connections": glob.n_conns if scaling == "strong" else glob.n_conns * world,
                   "global_payload_bytes": glob.payload_len if scaling == "strong" else None,
                   "parallelism": (f"connections sharded over {world} GPU(s)"
                                   f"{' by greedy LPT over stream bytes' if scaling == 'strong' else ''}; "
                                   f"{'RCCL' if dist.backend() == 'nccl' else dist.backend()} all-reduce of counts"),
                   "batches_in_flight": M,
                   **({"input_mem": args.input_mem} if args.input_mem != "default" else {}),
                   **({"emulated_shard": emulated} if emulated else {})},
        "frames_per_s": round(frames_step * args.steps / elapsed, 1),
        "decoded_per_step": {"frames": frames_step, "payload_bytes": payload_step, "errors": errors,
                             "ranks_summed": world},
        "errors": errors,
        "walk": walk_info,
        "phases_ms": {"walk_count": round(mean_ms[0], 4), "scan": round(mean_ms[1], 4),
                      "walk_emit": round(mean_ms[2], 4), "unmask": round(unmask_ms, 4)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "k_unmask", "algorithmic_bytes_per_launch": alg_bytes,
                     "pipeline_achieved": round(pipeline_gbps, 1),
                     "pipeline_frac": round(pipeline_gbps / HBM_PEAK_GBPS, 4),
                     "copy_ceiling": None if copy_gbps is None else round(copy_gbps, 1),
                     "copy_ceiling_by_load": copy_by_load or None,
                     "frac_of_copy_ceiling": None if copy_gbps is None else round(achieved / copy_gbps, 4),
                     **({"copy_interleaved": interleaved} if interleaved else {})},
        "verified_bit_exact": True,
        "frame_size_histogram": (size_histogram(glob) if args.config in ("c4", "c5") else None),
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu:
        log("cpu baseline (1 thread)...")
        result["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds, 1)
        nt = args.cpu_threads_multi or all_host_threads()
        if nt > 1:
            log(f"cpu baseline ({nt} threads)...")
            result["cpu_baseline_multi"] = cpu_baseline(args.config, max(args.cpu_seconds / 2, 1.0), nt)
        quota = host_cpu_info()["cgroup_cpu_quota"]
        if not args.cpu_threads_multi and quota and 1 < math.ceil(quota) < nt:
            # the job's CPU share is capped below its visible threads: also time
            # one thread per CPU of the quota (no time-sharing between threads)
            nq = math.ceil(quota)
            log(f"cpu baseline ({nq} threads = cgroup quota)...")
            result["cpu_baseline_quota"] = cpu_baseline(args.config, max(args.cpu_seconds / 2, 1.0), nq)
        log("cpu baseline (1 thread, auto-vectorised build)...")
        result["cpu_baseline_vectorized"] = cpu_baseline(args.config, max(args.cpu_seconds / 2, 1.0), 1,
                                                         vectorized=True)
        # the same pipeline with make() recycling one cache-warm chunk (calloc /
        # free): the flattering variant, beside the fresh-memory legs above
        log("cpu baseline (1 thread, cache-hot allocation)...")
        result["cpu_baseline_cache_hot"] = cpu_baseline(args.config, max(args.cpu_seconds / 2, 1.0), 1,
                                                        alloc="cache_hot")
        if "cpu_baseline_quota" in result:
            log(f"cpu baseline ({nq} threads, cache-hot allocation)...")
            result["cpu_baseline_quota_cache_hot"] = cpu_baseline(args.config, max(args.cpu_seconds / 2, 1.0), nq,
                                                                  alloc="cache_hot")
    print(json.dumps(result), flush=True)
    dist.finalize()


if __name__ == "__main__":
    main()
