"""N > 1 path on the CPU: two ranks over gloo run the same sharding and
collective code the bench runs over RCCL (gev_amd/dist.py), with each rank's
decode done by the oracle.  Checks that the connection -> rank split covers
every connection exactly once, that the summed counts equal the whole batch's,
and the max-over-ranks timing reduce."""
import json
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import torch
    from gev_amd import dist, workloads as w
    from oracle import ref
    dist.init("gloo")
    res = {}
    # strong scaling: one global batch, connections split byte-balanced
    glob = w.config_c5(n_conns=7, messages_per_conn=1, message_bytes=48 * 1024, seed=3)
    part = w.shard(glob, rank, world)
    arena = np.concatenate([w.synth_host(part), np.zeros(64, np.uint8)])
    r = ref.decode_batch(arena, part.conns[:, 0], part.conns[:, 1])
    counts = torch.tensor([r["frames"].shape[0], int(r["frames"]["length"].sum()),
                           int((r["conn_status"] < 0).sum())], dtype=torch.int64)
    dist.reduce_counts(counts)
    res["strong"] = counts.tolist()
    res["strong_conns"] = part.n_conns
    # the bench's C4 strong split: greedy LPT over stream bytes (workloads.shard_lpt)
    glob4 = w.config_c4(total_payload=3 << 20, n_conns=23, seed=13)
    part = w.shard_lpt(glob4, rank, world)
    arena = np.concatenate([w.synth_host(part), np.zeros(64, np.uint8)])
    r = ref.decode_batch(arena, part.conns[:, 0], part.conns[:, 1])
    counts = torch.tensor([r["frames"].shape[0], int(r["frames"]["length"].sum()),
                           int((r["conn_status"] < 0).sum())], dtype=torch.int64)
    dist.reduce_counts(counts)
    res["lpt"] = counts.tolist()
    res["lpt_conns"] = part.n_conns
    res["lpt_max_bytes"] = dist.max_over_ranks(float(part.arena_bytes), "cpu")
    # weak scaling: every rank its own same-shape batch
    lay = w.uniform(3, 4, 1000, seed=dist.rank_seed(5, rank))
    arena = np.concatenate([w.synth_host(lay), np.zeros(64, np.uint8)])
    r = ref.decode_batch(arena, lay.conns[:, 0], lay.conns[:, 1])
    counts = torch.tensor([r["frames"].shape[0], int(r["frames"]["length"].sum()), 0], dtype=torch.int64)
    dist.reduce_counts(counts)
    res["weak"] = counts.tolist()
    res["max"] = dist.max_over_ranks(float(rank + 1), "cpu")
    dist.barrier()
    dist.finalize()
    json.dump(res, open(os.path.join(outdir, f"r{rank}.json"), "w"))


@pytest.mark.parametrize("world", [2])
def test_gloo_shard_and_count_reduce(tmp_path, world):
    import torch.multiprocessing as mp
    from gev_amd import workloads as w
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    res = [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]
    glob = w.config_c5(n_conns=7, messages_per_conn=1, message_bytes=48 * 1024, seed=3)
    glob4 = w.config_c4(total_payload=3 << 20, n_conns=23, seed=13)
    lens4 = glob4.conns[:, 1]
    for r in res:
        assert r["strong"] == [glob.n_frames, glob.payload_len, 0]
        assert r["lpt"] == [glob4.n_frames, glob4.payload_len, 0]
        assert r["lpt_max_bytes"] <= 4 / 3 * max(lens4.sum() / world, lens4.max()) + 1  # Graham's bound
        assert r["weak"] == [world * 12, world * 12 * 1000, 0]
        assert r["max"] == float(world)
    assert sum(r["strong_conns"] for r in res) == glob.n_conns
    assert sum(r["lpt_conns"] for r in res) == glob4.n_conns


def test_shard_bounds_partition_and_balance():
    from gev_amd import workloads as w
    rng = np.random.default_rng(0)
    for _ in range(200):
        n = int(rng.integers(0, 50))
        lens = rng.integers(0, 10_000, n)
        for world in (1, 2, 3, 4, 8):
            b = w.shard_bounds(lens, world)
            assert b[0] == 0 and b[-1] == n and len(b) == world + 1
            assert all(b[i] <= b[i + 1] for i in range(world))
            if n and lens.sum():
                share = lens.sum() / world
                for r in range(world):
                    got = lens[b[r]:b[r + 1]].sum()
                    assert got <= share + lens.max() + 1


def test_shard_layouts_reassemble():
    from gev_amd import workloads as w
    lay = w.config_c4(total_payload=2 << 20, n_conns=16, seed=9)
    parts = [w.shard(lay, r, 4) for r in range(4)]
    assert sum(p.n_frames for p in parts) == lay.n_frames
    assert sum(p.payload_len for p in parts) == lay.payload_len
    assert sum(p.arena_bytes for p in parts) == lay.arena_bytes
    assert np.array_equal(np.concatenate([p.desc["length"] for p in parts]), lay.desc["length"])


def test_lpt_shard_partition_and_balance():
    from gev_amd import workloads as w
    lay = w.config_c4(total_payload=4 << 20, n_conns=37, seed=11)
    lens = lay.conns[:, 1]
    for world in (1, 2, 3, 8):
        parts = [w.shard_lpt(lay, r, world) for r in range(world)]
        assert sum(p.n_frames for p in parts) == lay.n_frames
        assert sum(p.payload_len for p in parts) == lay.payload_len
        assert sum(p.arena_bytes for p in parts) == lay.arena_bytes
        assert sorted(np.concatenate([p.conns[:, 1] for p in parts]).tolist()) == sorted(lens.tolist())
        # Graham's bound for greedy LPT
        assert max(p.arena_bytes for p in parts) <= 4 / 3 * max(lens.sum() / world, lens.max()) + 1
        for p in parts:
            # each rank's arena is a valid back-to-back layout: frames tile every stream exactly
            h = w.header_len(p.desc["length"].astype(np.int64), p.desc["masked"], p.desc["len_form"].astype(np.int64))
            end = p.desc["hdr_off"].astype(np.int64) + h + p.desc["length"].astype(np.int64)
            assert np.array_equal(end[:-1], p.desc["hdr_off"][1:].astype(np.int64))
            if p.n_conns:
                assert np.array_equal(p.conns[1:, 0], (p.conns[:, 0] + p.conns[:, 1])[:-1])


def test_lpt_shard_decodes_to_global_frames():
    """The frames every rank decodes (oracle) are exactly the global batch's frames."""
    from gev_amd import workloads as w
    from oracle import ref
    lay = w.config_c5(n_conns=6, messages_per_conn=1, message_bytes=20 * 1024, seed=4)
    got = []
    for r in range(3):
        p = w.shard_lpt(lay, r, 3)
        if p.n_conns == 0:
            continue
        arena = np.concatenate([w.synth_host(p), np.zeros(64, np.uint8)])
        d = ref.decode_batch(arena, p.conns[:, 0], p.conns[:, 1])
        assert (d["conn_status"] >= 0).all() and d["frames"].shape[0] == p.n_frames
        got += list(zip(d["frames"]["length"].tolist(), d["frames"]["opcode"].tolist()))
    want = list(zip(lay.desc["length"].tolist(), (lay.desc["b0"] & 0xF).tolist()))
    assert sorted(got) == sorted(want)


def test_size_histogram_counts_every_frame():
    from gev_amd import workloads as w
    lay = w.config_c5(n_conns=4, messages_per_conn=1, message_bytes=30 * 1024, seed=2)
    hist = w.size_histogram(lay)
    assert sum(c for _, _, c in hist) == lay.n_frames
    for lo, hi, c in hist:
        m = (lay.desc["length"] >= lo) & (lay.desc["length"] <= hi)
        assert int(m.sum()) == c
