"""GPU parity suite: the HIP decode path, called through the C ABI, against the
oracle and the golden vectors -- bit-exact (integer/byte work, no tolerance).

Small and medium batches are compared record by record and byte by byte with
oracle/ws_ref.c; full BASELINE sizes (C2, C3) are checked with the
size-independent property decode(mask(P)) == P on the device generator's
frames (gevws_synth_verify_async), plus an oracle cross-check of a slice."""
import numpy as np
import pytest

import gev_amd
from oracle import ref
from oracle import ws_oracle as wo
from tests._helpers import assert_matches_oracle, gpu_decode, host_result, pack_streams, random_stream

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["one_launch", "multi_kernel"])
def small_path(engine, request):
    """Small batches run the one-launch decode (k_decode_small) by default;
    the multi-kernel path (walk, scan, records, unmask) must give the same
    bytes, so the core parity tests run both."""
    from gev_amd import _abi
    engine.set_tuning(_abi.TUNE_SMALL_BATCH, _abi.ONE_LAUNCH_MAX_BYTES if request.param == "one_launch" else 0)
    yield request.param
    engine.set_tuning(_abi.TUNE_SMALL_BATCH, _abi.ONE_LAUNCH_MAX_BYTES)


# --------------------------------------------------------------------------- golden vectors
def test_golden_vectors(engine, golden, small_path):
    for name, g in golden.items():
        if name == "encode":
            continue  # tests/test_gpu_encode.py
        got = host_result(gpu_decode(engine, g["in"], g["conns"]))
        co = got["conn_out"]
        assert np.array_equal(co["nframes"], g["conn_res"][:, 0]), name
        assert np.array_equal(co["consumed"], g["conn_res"][:, 1]), name
        assert np.array_equal(co["status"], g["conn_res"][:, 2]), name
        f = got["frames"]
        assert np.array_equal(f.view(np.uint8).reshape(-1, 32)[:, :16], g["hdr"]), name
        assert np.array_equal(f["src_off"], g["src_off"]), name
        pay = got["payload"]
        cat = b"".join(pay[int(o):int(o) + int(L)].tobytes() for o, L in zip(f["payload_off"], f["length"]))
        assert cat == g["payload"].tobytes(), name
        assert_matches_oracle(engine, g["in"], g["conns"], name)


def test_rfc6455_kats_on_device(engine, small_path):
    arena = b"".join(k[0] for k in wo.RFC6455_KATS)
    got = host_result(gpu_decode(engine, arena, np.array([[0, len(arena)]])))
    assert int(got["summary"]["frames"]) == len(wo.RFC6455_KATS)
    for f, k in zip(got["frames"], wo.RFC6455_KATS):
        o, L = int(f["payload_off"]), int(f["length"])
        assert got["payload"][o:o + L].tobytes() == k[5]


# --------------------------------------------------------------------------- alignment / edge sweeps
def test_alignment_and_length_sweep(engine, small_path):
    """Every payload start mod 16 x every length class near the 16-byte chunk edges."""
    rng = np.random.default_rng(11)
    streams = []
    lengths = list(range(0, 70)) + [k * 16 + d for k in (5, 8, 63, 64, 256) for d in (-1, 0, 1)] + [4093, 4096, 4099]
    for lead in range(16):
        s = bytes(rng.integers(0, 256, lead, dtype=np.uint8))  # garbage prefix consumed as its own conn
        streams.append(s)
        body = b""
        for L in lengths:
            body += wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), 2, True, 0,
                                    bool(L % 3), bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
        streams.append(body + b"\x00" * 6)
    arena, conns = pack_streams(streams)
    assert_matches_oracle(engine, arena, conns, "alignment sweep")


def test_random_batches(engine, small_path):
    rng = np.random.default_rng(12)
    for trial in range(6):
        n = int(rng.integers(1, 300))
        streams = [random_stream(rng, int(rng.integers(0, 25))) for _ in range(n)]
        arena, conns = pack_streams(streams)
        assert_matches_oracle(engine, arena, conns, f"trial {trial}")


def test_unordered_and_overlapping_conn_tables(engine, small_path):
    """the walk's per-connection entry runs are placed by
    input offset, which is collision-free only for a table in increasing,
    non-overlapping order.  Tables that break it -- the advisor's example
    (neighbour checks all pass for conn 0 and conn 3, whose runs collide),
    shuffled, reversed and overlapping tables -- must decode exactly as the
    oracle decodes the same table, and report GEVWS_SUMMARY_UNORDERED."""
    rng = np.random.default_rng(15)
    s0 = b"".join(wo.encode_frame(bytes(rng.integers(0, 256, 190, dtype=np.uint8)), 2, True, 0, True,
                                  bytes(rng.integers(0, 256, 4, dtype=np.uint8))) for _ in range(20))
    arena = s0 + bytes(rng.integers(0, 256, 5010 - len(s0), dtype=np.uint8))
    conns = np.array([[0, len(s0)], [5000, 10], [50, 10], [60, 30]], np.int64)
    got = assert_matches_oracle(engine, arena, conns, "advisor example")
    assert int(got["summary"]["flags"]) & gev_amd.SUMMARY_UNORDERED
    for trial in range(4):
        streams = [random_stream(rng, int(rng.integers(0, 30)), max_len=600) for _ in range(int(rng.integers(40, 400)))]
        arena, conns = pack_streams(streams)
        got = assert_matches_oracle(engine, arena, conns, f"ordered {trial}")
        assert int(got["summary"]["flags"]) == 0
        perm = rng.permutation(conns.shape[0]) if trial % 2 == 0 else np.arange(conns.shape[0])[::-1]
        got = assert_matches_oracle(engine, arena, conns[perm], f"permuted {trial}")
        assert int(got["summary"]["flags"]) & gev_amd.SUMMARY_UNORDERED
    # overlapping streams (the same bytes decoded twice) and a 4-fold repeat
    arena, conns = pack_streams([random_stream(rng, 25, max_len=900) for _ in range(64)])
    assert_matches_oracle(engine, arena, np.concatenate([conns, conns[::3]]), "overlap")
    assert_matches_oracle(engine, arena, np.tile(conns, (4, 1)), "repeat")


def test_random_garbage_streams(engine, small_path):
    """Streams of random bytes (headers parsed from noise: 16- and 64-bit length
    codes, MSB-set lengths, incomplete payloads, short tails), alone and behind
    a few valid frames, decode exactly as the oracle decodes them."""
    rng = np.random.default_rng(14)
    for trial in range(4):
        streams = []
        for _ in range(int(rng.integers(50, 400))):
            # noise: len7 is <= 125 for most second bytes, so many noise
            # "frames" complete; 127-codes carry random 64-bit lengths (MSB set
            # half the time -> ErrHeaderLengthMSB)
            junk = bytes(rng.integers(0, 256, int(rng.integers(0, 4000)), dtype=np.uint8))
            lead = random_stream(rng, int(rng.integers(0, 4)), max_len=300, tail=False) if rng.random() < 0.5 else b""
            streams.append(lead + junk)
        arena, conns = pack_streams(streams)
        assert_matches_oracle(engine, arena, conns, f"garbage trial {trial}")


def test_big_frames_cross_tiles(engine, small_path):
    rng = np.random.default_rng(13)
    s = b""
    for L in (1 << 20, 65536, 70001, 4096 * 3 + 5, 1, 0, (1 << 20) + 17):
        s += wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), 2, True, 0, True,
                             bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
    arena, conns = pack_streams([s, s[:-3], s[5:]])
    assert_matches_oracle(engine, arena, conns, "big frames")


def test_empty_and_tiny_batches(engine, small_path):
    assert_matches_oracle(engine, b"", np.zeros((0, 2), np.int64), "no conns")
    assert_matches_oracle(engine, b"\x81", np.array([[0, 1], [1, 0]]), "1 byte + empty")
    arena, conns = pack_streams([b"", b"\x81\x00", b"\x81\x80\x01\x02\x03\x04"])
    assert_matches_oracle(engine, arena, conns, "tiny")


def test_poisoned_connections_isolated(engine, small_path):
    good = wo.encode_frame(b"fine", 1, True, 0, True, b"\x01\x02\x03\x04")
    bad = bytes([0x82, 0xFF, 0x80, 0, 0, 0, 0, 0, 0, 5, 1, 2, 3, 4]) + b"hello"
    arena, conns = pack_streams([good + bad + good, good * 3, bad, good])
    got = assert_matches_oracle(engine, arena, conns, "poison")
    assert list(got["conn_out"]["status"]) == [-1, 0, -1, 0]
    assert int(got["summary"]["errors"]) == 2


def test_streams_outside_the_arena_are_rejected(engine, small_path):
    """A connection whose [off, off + len) leaves the input arena reads nothing
    and reports GEVWS_ERR_INVALID; the connections around it decode exactly as
    the oracle decodes them on their own."""
    import gev_amd
    good = [wo.encode_frame(b"abc" * k, 2, True, 0, True, b"\x01\x02\x03\x04") * 3 for k in (1, 50, 400)]
    arena, conns = pack_streams(good)
    n = len(arena)
    bad = np.array([[n - 4, 10], [n + 100, 5], [1 << 62, 1 << 62]], np.int64)
    table = np.concatenate([conns[:1], bad[:1], conns[1:2], bad[1:], conns[2:]])
    got = host_result(gpu_decode(engine, arena, table))
    st = got["conn_out"]["status"]
    assert list(st) == [0, gev_amd.ERR_INVALID, 0, gev_amd.ERR_INVALID, gev_amd.ERR_INVALID, 0]
    assert int(got["summary"]["errors"]) == 3
    assert list(got["conn_out"]["nframes"][[1, 3, 4]]) == [0, 0, 0]
    assert list(got["conn_out"]["consumed"][[1, 3, 4]]) == [0, 0, 0]
    want = ref.decode_batch(np.frombuffer(arena, np.uint8).copy(), conns[:, 0], conns[:, 1])
    assert got["frames"].tobytes() == want["frames"].tobytes()
    assert np.array_equal(got["payload"], want["payload"])


def test_decode_into_mapped_host_arena(engine, small_path):
    """The payload arena may be mapped pinned host memory (gevws_pinned_alloc):
    the unmask kernel's writes land in host pages, byte-identical to the oracle,
    and the bytes past the arena stay untouched."""
    import torch
    import gev_amd
    rng = np.random.default_rng(21)
    s = b"".join(wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), 2, True, 0, True,
                                 bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
                 for L in (70001, 3, 0, 4096 * 5 + 9, 125, 65536))
    arena, conns = pack_streams([random_stream(rng, 30), s, s[7:], random_stream(rng, 5)])
    a = np.frombuffer(arena, np.uint8).copy()
    want = ref.decode_batch(a, conns[:, 0], conns[:, 1])
    cap = int(want["total_payload"])
    dev = torch.device("cuda", engine.device)
    d_in = torch.zeros(a.size + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    d_in[: a.size] = torch.from_numpy(a).to(dev)
    d_conns = torch.from_numpy(conns.copy()).to(dev)
    host = gev_amd.PinnedArena(cap + 4096)
    try:
        host.host[:] = 0xA5
        o = engine.alloc_batch(conns.shape[0], want["frames"].shape[0], 0)
        out = gev_amd.Batch(frames=o.frames, payload=host.at(0), conn_out=o.conn_out, summary=o.summary,
                            n_conns=o.n_conns)
        engine.decode_async(d_in, a.size, d_conns, conns.shape[0], out, want["frames"].shape[0], cap)
        torch.cuda.synchronize()
        sm = o.summary.cpu().numpy().view(gev_amd.SUMMARY_DTYPE)[0]
        assert int(sm["status"]) == 0 and int(sm["payload_bytes"]) == cap
        assert o.frames.cpu().numpy().tobytes() == want["frames"].tobytes()
        assert np.array_equal(host.host[:cap], want["payload"])
        assert (host.host[cap:] == 0xA5).all()
    finally:
        host.close()


def test_capacity_error_reports_exact_sizes(engine, small_path):
    import torch
    rng = np.random.default_rng(14)
    arena, conns = pack_streams([random_stream(rng, 20, tail=False) for _ in range(10)])
    want = ref.decode_batch(np.frombuffer(arena, np.uint8).copy(), conns[:, 0], conns[:, 1])
    import gev_amd
    dev = torch.device("cuda", engine.device)
    d_in = torch.zeros(len(arena) + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    d_in[: len(arena)] = torch.from_numpy(np.frombuffer(arena, np.uint8).copy()).to(dev)
    d_conns = torch.from_numpy(conns.copy()).to(dev)
    out = engine.alloc_batch(conns.shape[0], 5, 64)
    engine.decode_async(d_in, len(arena), d_conns, conns.shape[0], out, 5, 64)
    torch.cuda.synchronize()
    s = out.summary_host()
    assert int(s["status"]) == gev_amd.ERR_CAPACITY
    assert int(s["frames"]) == want["frames"].shape[0]
    assert int(s["payload_bytes"]) == want["total_payload"]
    # the retrying wrapper then succeeds
    assert_matches_oracle(engine, arena, conns, "after capacity retry")


# --------------------------------------------------------------------------- ws.Cipher on device
def test_device_cipher_all_offsets_alignments(engine):
    import torch
    rng = np.random.default_rng(15)
    base = rng.integers(0, 256, 70000, dtype=np.uint8)
    dev = torch.device("cuda", engine.device)
    for n in list(range(0, 40)) + [63, 64, 65, 1000, 4097, 65536]:
        for align in (0, 1, 3, 7, 8, 13, 15):
            for off in range(0, 8):
                mask = bytes(rng.integers(0, 256, 4, dtype=np.uint8))
                t = torch.from_numpy(base[:align + n + 16].copy()).to(dev)
                engine.cipher_(t, mask, off, nbytes=n, byte_offset=align)
                got = t.cpu().numpy()
                want = base[:align + n + 16].copy()
                c = want[align:align + n]
                ref.cipher(c, mask, off)
                want[align:align + n] = c
                assert np.array_equal(got, want), (n, align, off)


# --------------------------------------------------------------------------- synthetic full-size properties
def _synth_decode_verify(engine, layout, check_slice_conns: int = 2):
    import torch
    import gev_amd
    dev = torch.device("cuda", engine.device)
    arena = torch.empty(layout.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    arena[layout.arena_bytes:] = 0
    desc = torch.from_numpy(layout.desc.view(np.uint8).copy()).to(dev)
    conns = torch.from_numpy(layout.conns.copy()).to(dev)
    engine.synth(arena, desc, layout.n_frames, layout.seed)
    out = engine.decode(arena, layout.arena_bytes, conns, layout.n_conns, max_frames=layout.n_frames,
                        payload_cap=layout.payload_padded)
    s = out.summary_host()
    assert int(s["frames"]) == layout.n_frames
    assert int(s["payload_len"]) == layout.payload_len
    from gev_amd import workloads as wl
    assert int(s["run_frames"]) == wl.run_frames(layout)
    assert int(s["payload_bytes"]) == layout.payload_padded
    mism = torch.zeros(1, dtype=torch.int64, device=dev)
    engine.verify(desc, layout.n_frames, layout.seed, out, mism)
    torch.cuda.synchronize()
    assert int(mism.item()) == 0
    co = out.conn_out_host()
    assert np.array_equal(co["consumed"].astype(np.int64), layout.conns[:, 1])
    # oracle cross-check of the first connections' streams, byte for byte
    k = min(check_slice_conns, layout.n_conns)
    end = int(layout.conns[k - 1, 0] + layout.conns[k - 1, 1])
    host_in = arena[:end].cpu().numpy()
    want = ref.decode_batch(host_in, layout.conns[:k, 0], layout.conns[:k, 1])
    nf = want["frames"].shape[0]
    got_frames = out.frames[:nf].cpu().numpy().reshape(-1).view(want["frames"].dtype)
    assert got_frames.tobytes() == want["frames"].tobytes()
    got_pay = out.payload[: want["total_payload"]].cpu().numpy()
    assert np.array_equal(got_pay, want["payload"])
    # and the generator's plaintext on the host for frame 0
    from gev_amd import workloads
    L0 = int(layout.desc["length"][0])
    assert got_pay[:L0].tobytes() == workloads.plaintext(layout.seed, 0, L0)
    del arena, out
    torch.cuda.empty_cache()


def test_c2_full_size_property(engine):
    from gev_amd import workloads
    _synth_decode_verify(engine, workloads.config_c2())


def test_c3_full_size_property(engine):
    import torch
    from gev_amd import workloads
    lay = workloads.config_c3()
    free, _ = torch.cuda.mem_get_info(engine.device)
    need = lay.arena_bytes + lay.payload_padded + (1 << 30)
    if free < need:
        pytest.fail(f"C3 needs {need / 2**30:.1f} GiB of HBM, {free / 2**30:.1f} GiB free")
    _synth_decode_verify(engine, lay, check_slice_conns=1)


def test_stream_over_4gib_and_small_frame_fallback(engine):
    """A connection whose buffered stream exceeds 4 GiB (32-bit walk entries
    cannot hold its offsets: the emit pass re-walks it) next to connections of
    10-byte frames (more frames than entry slots: re-walked too) and ordinary
    ones, in one batch: decode(mask(P)) == P on every byte."""
    import numpy as np
    from gev_amd import workloads as w
    big = w.uniform(1, 65600, 65536, seed=5)  # 4.3 GB stream, h = 14
    small = w.uniform(64, 500, 4, seed=6)
    mid = w.uniform(8, 40, 3000, seed=7)
    parts = [small, big, mid]
    desc, conns, off = [], [], 0
    for lay in parts:
        d = lay.desc.copy()
        d["hdr_off"] += np.uint64(off)
        desc.append(d)
        c = lay.conns.copy()
        c[:, 0] += off
        conns.append(c)
        off += lay.arena_bytes
    desc = np.concatenate(desc)
    desc["mask"] = w.frame_masks(desc.shape[0], 11)
    lay = w.Layout("4 GiB stream + tiny frames", desc, np.concatenate(conns), off,
                   sum(p.payload_len for p in parts), sum(p.payload_padded for p in parts), 11)
    assert lay.conns[64, 1] > 1 << 32
    _synth_decode_verify(engine, lay, check_slice_conns=8)


def _oracle_compare_conns(engine, out, arena, layout, idx):
    """Byte-compare the device result of the connections `idx` (any subset of
    the batch) with the oracle: their streams are copied to the host, decoded
    by oracle/ws_ref.c as a batch of their own, and every record / payload
    byte is compared after rebasing offsets (input offsets by the stream's
    position, payload offsets by the connection's arena base)."""
    idx = np.asarray(idx, np.int64)
    co = out.conn_out_host()
    streams = [arena[int(layout.conns[c, 0]):int(layout.conns[c, 0] + layout.conns[c, 1])].cpu().numpy() for c in idx]
    lens = np.array([x.size for x in streams], np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    want = ref.decode_batch(np.concatenate(streams + [np.zeros(64, np.uint8)]), offs, lens)
    wf = want["frames"]
    for j, c in enumerate(idx):
        n = int(co["nframes"][c])
        assert n == int(want["conn_nframes"][j]) and int(co["consumed"][c]) == int(want["conn_consumed"][j]), c
        assert int(co["status"][c]) == int(want["conn_status"][j]), c
        f0, w0 = int(co["first_frame"][c]), int(want["conn_first"][j])
        g = out.frames[f0:f0 + n].cpu().numpy().reshape(-1).view(wf.dtype)
        w = wf[w0:w0 + n]
        assert g.view(np.uint8).reshape(-1, 32)[:, :16].tobytes() == w.view(np.uint8).reshape(-1, 32)[:, :16].tobytes(), c
        gb, wb = int(co["payload_base"][c]), int(w["payload_off"][0]) if n else 0
        assert np.array_equal(g["payload_off"] - np.uint64(gb), w["payload_off"] - np.uint64(wb)), c
        assert np.array_equal(g["src_off"] - np.uint64(layout.conns[c, 0]), w["src_off"] - np.uint64(offs[j])), c
        if n:
            end = int(w["payload_off"][-1]) + (int(w["length"][-1]) + 15) // 16 * 16 - wb
            gp = out.payload[gb:gb + end].cpu().numpy()
            assert np.array_equal(gp, want["payload"][wb:wb + end]), c
    return int(wf.shape[0])


def _c4_full(engine, lay, n_check: int = 64, expect_split=None):
    """BASELINE config 4 at its configured size (or an LPT share of it): every
    byte by the generator property, plus >= n_check connections -- the longest
    chain among them -- byte-compared with the oracle."""
    import torch
    import gev_amd
    dev = torch.device("cuda", engine.device)
    free, _ = torch.cuda.mem_get_info(engine.device)
    need = lay.arena_bytes + lay.payload_padded + lay.n_frames * 32 + lay.arena_bytes // 4 + (2 << 30)
    if free < need:
        pytest.fail(f"{lay.name}: needs {need / 2**30:.1f} GiB of HBM, {free / 2**30:.1f} GiB free")
    arena = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    arena[lay.arena_bytes:] = 0
    desc = torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev)
    conns = torch.from_numpy(lay.conns.copy()).to(dev)
    engine.synth(arena, desc, lay.n_frames, lay.seed)
    out = engine.decode(arena, lay.arena_bytes, conns, lay.n_conns, max_frames=lay.n_frames,
                        payload_cap=lay.payload_padded)
    s = out.summary_host()
    if expect_split is not None:  # which header walk ran (k_walk_split: lanes per connection)
        assert engine.last_split_lanes == expect_split, (lay.name, engine.last_split_lanes)
    assert int(s["frames"]) == lay.n_frames and int(s["payload_len"]) == lay.payload_len
    assert int(s["payload_bytes"]) == lay.payload_padded and int(s["errors"]) == 0 and int(s["flags"]) == 0
    from gev_amd import workloads as wl
    assert int(s["run_frames"]) == wl.run_frames(lay)
    mism = torch.zeros(1, dtype=torch.int64, device=dev)
    engine.verify(desc, lay.n_frames, lay.seed, out, mism)
    torch.cuda.synchronize()
    assert int(mism.item()) == 0
    counts = np.diff(np.searchsorted(lay.desc["hdr_off"].astype(np.int64),
                                     np.concatenate([lay.conns[:, 0], [lay.arena_bytes]])))
    longest = int(np.argmax(counts))
    rng = np.random.default_rng(4)
    idx = np.unique(np.concatenate([[0, longest, lay.n_conns - 1],
                                    rng.choice(lay.n_conns, min(n_check, lay.n_conns), replace=False)]))
    nf = _oracle_compare_conns(engine, out, arena, lay, idx)
    del arena, out, desc
    torch.cuda.empty_cache()
    return int(counts[longest]), nf, idx.size


def test_c4_full_size_and_lpt_shards(engine):
    """BASELINE config 4 exactly as bench.py builds it (16 GiB power-law
    payload over 65 536 connections, 43.8 M frames) on one GPU, then rank 0's
    and rank 7's greedy-LPT shares of the 8-way strong split and rank 0's of
    the 4-way."""
    import torch
    import bench
    from gev_amd import workloads as w
    glob, _ = bench.build_layout("c4", 0, None)
    assert glob.payload_len >= 16 << 30 and glob.n_conns == 65536
    longest, nf, k = _c4_full(engine, glob, expect_split=1)
    assert longest > 1000 and k >= 64 and nf > 0
    # the 8-way shares after the full batch: the auto choice splits their walk
    # (16 lanes per connection, k_walk_split) on the full batch's history
    for r in (0, 7):
        part = w.shard_lpt(glob, r, 8)
        assert part.n_conns == 65536 // 8 or abs(part.n_conns - 65536 // 8) < 65536 // 16
        ncu = torch.cuda.get_device_properties(engine.device).multi_processor_count
        _c4_full(engine, part, expect_split=16 if part.n_conns <= 32 * ncu else None)
    # rank 0's 4-way share (64 connections per CU): split 8 ways since round 6
    # (entries through the writer wave, profiles/r06/r06i_split_rule.jsonl)
    part = w.shard_lpt(glob, 0, 4)
    _c4_full(engine, part, expect_split=8 if part.n_conns <= 64 * ncu else None)


def test_c4_power_law_property(engine):
    from gev_amd import workloads
    _synth_decode_verify(engine, workloads.config_c4(total_payload=64 << 20, n_conns=512), check_slice_conns=8)


def test_c5_fragmented_control_property(engine):
    from gev_amd import workloads
    lay = workloads.config_c5(n_conns=16, messages_per_conn=2)
    _synth_decode_verify(engine, lay, check_slice_conns=16)


def test_device_generator_matches_host_generator(engine):
    """The device frame generator (bench / full-size property tests) writes
    exactly the bytes of workloads.synth_host, so the oracle-checked slices
    above stand for the whole batch's format."""
    import torch
    import gev_amd
    from gev_amd import workloads as w
    dev = torch.device("cuda", engine.device)
    for lay in (w.uniform(3, 5, 4096 + 7, seed=11), w.config_c5(n_conns=3, messages_per_conn=1, seed=12),
                w.config_c4(total_payload=1 << 20, n_conns=4, seed=13)):
        arena = torch.zeros(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
        desc = torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev)
        engine.synth(arena, desc, lay.n_frames, lay.seed)
        torch.cuda.synchronize()
        assert np.array_equal(arena[: lay.arena_bytes].cpu().numpy(), w.synth_host(lay)), lay.name


def test_small_frame_window_paths(engine):
    """The unmask kernel's LDS window path (<= 1024 frames per 16 KiB window)
    and its fallback (more frames than that: runs of empty frames, 16-byte
    frames), mixed with frames that straddle windows."""
    rng = np.random.default_rng(16)
    m = bytes(rng.integers(0, 256, 4, dtype=np.uint8))
    tiny16 = b"".join(wo.encode_frame(bytes(rng.integers(0, 256, 16, dtype=np.uint8)), 2, True, 0, True, m)
                      for _ in range(2500))
    tiny_mixed = b"".join(wo.encode_frame(bytes(rng.integers(0, 256, int(rng.integers(0, 17)), dtype=np.uint8)),
                                          2, True, 0, bool(rng.random() < .8), m) for _ in range(3000))
    empties = b"".join(wo.encode_frame(b"", 9, True, 0, True, m) for _ in range(3000))
    big = wo.encode_frame(bytes(rng.integers(0, 256, 50000, dtype=np.uint8)), 2, True, 0, True, m)
    mid = b"".join(wo.encode_frame(bytes(rng.integers(0, 256, int(rng.integers(100, 9000)), dtype=np.uint8)),
                                   1, True, 0, True, m) for _ in range(40))
    streams = [tiny16, big + empties + big, tiny_mixed + mid, mid + tiny16[:5000] + big, empties]
    arena, conns = pack_streams(streams)
    assert_matches_oracle(engine, arena, conns, "small-frame windows")


def test_one_context_two_streams_is_ordered(engine):
    """A context's scratch is shared by its calls: a call on another stream is
    ordered after the previous one (gevws_ctx semantics), so two batches
    issued back to back on two streams through ONE context both decode right."""
    import torch
    import gev_amd
    rng = np.random.default_rng(17)
    dev = torch.device("cuda", engine.device)
    batches = []
    for nconn in (200, 37):
        streams = [random_stream(rng, int(rng.integers(0, 40))) for _ in range(nconn)]
        arena, conns = pack_streams(streams)
        a = np.frombuffer(arena, np.uint8).copy()
        d_in = torch.zeros(a.size + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
        d_in[: a.size] = torch.from_numpy(a).to(dev)
        d_c = torch.from_numpy(conns.copy()).to(dev)
        mf, cap = a.size // 2 + 1, a.size * 9 + 64
        batches.append((a, conns, d_in, d_c, engine.alloc_batch(nconn, mf, cap), mf, cap))
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for (a, conns, d_in, d_c, out, mf, cap), s in zip(batches, (s1, s2)):
        engine.decode_async(d_in, a.size, d_c, conns.shape[0], out, mf, cap, stream=s)
    torch.cuda.synchronize()
    for a, conns, d_in, d_c, out, mf, cap in batches:
        want = ref.decode_batch(a, conns[:, 0], conns[:, 1])
        assert out.frames_host().tobytes() == want["frames"].tobytes()
        assert np.array_equal(out.payload_host(), want["payload"])


def test_own_stream_live_pass_then_other_stream_is_ordered(engine):
    """A one-launch call on the context's own stream leaves its last-call
    event to be recorded when first needed (mark_last_lazy): a live pass
    posted there (gevws_decode_batch_post, staged through the context's
    granules by up to 32 workgroups) and one issued right after it on a
    torch stream (the same granules) still run in order, so both decode
    right -- five times over."""
    import torch
    import gev_amd
    rng = np.random.default_rng(18)
    dev = torch.device("cuda", engine.device)
    flag = gev_amd.PinnedArena(4096)
    engine.set_completion_flag(flag, 64)
    try:
        for rep in range(5):
            batches = []
            for nconn in (200, 150):
                streams = [random_stream(rng, int(rng.integers(1, 6)), max_len=200) for _ in range(nconn)]
                arena, conns = pack_streams(streams)
                a = np.frombuffer(arena, np.uint8).copy()
                d_in = torch.zeros(a.size + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
                d_in[: a.size] = torch.from_numpy(a).to(dev)
                d_c = torch.from_numpy(conns.copy()).to(dev)
                mf, cap = a.size // 2 + 1, a.size * 9 + 64
                batches.append((a, conns, d_in, d_c, engine.alloc_batch(nconn, mf, cap), mf, cap))
            torch.cuda.synchronize()
            (a, conns, d_in, d_c, out, mf, cap), second = batches
            engine.decode_post(d_in, a.size, d_c, conns.shape[0], out, mf, cap)  # the context's stream
            s1 = torch.cuda.Stream(dev)
            a, conns, d_in, d_c, out, mf, cap = second
            engine.decode_async(d_in, a.size, d_c, conns.shape[0], out, mf, cap, stream=s1)
            torch.cuda.synchronize()
            for a, conns, d_in, d_c, out, mf, cap in batches:
                assert int(out.summary_host()["status"]) == 0, rep
                want = ref.decode_batch(a, conns[:, 0], conns[:, 1])
                assert out.frames_host().tobytes() == want["frames"].tobytes(), rep
                assert np.array_equal(out.payload_host(), want["payload"]), rep
    finally:
        engine.set_completion_flag(None)
        flag.close()


def test_every_unmask_variant_big_frames_all_alignments(engine):
    """Each unmask variant (the default's aligned-load streaming path included)
    over frames >= 16 tiles whose payloads start at all 16 source alignments,
    with odd lengths, unmasked frames and small frames between them, in
    several connections: bit-exact against the C oracle."""
    from gev_amd import _abi
    rng = np.random.default_rng(77)
    streams, pos = [], 0     # pos: absolute arena offset (the arena starts 256-aligned on the device)
    for c in range(4):
        s = b""
        for k in range(12):
            masked = k % 5 != 4
            h = 14 if masked else 10
            want = (3 * c + 5 * k) % 16        # target source alignment of this payload
            # a small unmasked frame (2 + n bytes) moves the next payload to `want`
            n = (want - (pos + len(s) + 2 + h)) % 16 + 16 * int(rng.integers(0, 3))
            s += wo.encode_frame(bytes(rng.integers(0, 256, n, dtype=np.uint8)), 1, True, 0, False, b"\0" * 4)
            L = int(rng.integers(16 * 4096, 3 * 16 * 4096)) + int(rng.integers(0, 16))
            s += wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), 2, True, 0, masked,
                                 bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
        streams.append(s)
        pos += len(s)
    arena, conns = pack_streams(streams)
    i = 0
    while engine.variant_name(i) is not None:
        engine.set_tuning(_abi.TUNE_UNMASK_VARIANT, i)
        try:
            got = assert_matches_oracle(engine, arena, conns, f"variant {i}")
        finally:
            engine.set_tuning(_abi.TUNE_UNMASK_VARIANT, 0)
        i += 1
    # the sweep covered every source alignment of a streamed payload
    f = got["frames"]
    big = f["length"] >= 16 * 4096
    assert len(set((f["src_off"][big] % 16).tolist())) == 16


@pytest.mark.gpu
def test_every_unmask_variant_small_frame_windows(engine):
    """Each unmask variant over the window paths: random mixed frames
    (0-3072 B, every header form, unmasked and masked) in many connections, a
    run of 3000 empty frames between payloads (more frames per window than the
    LDS table holds), and 20 000 small frames in one connection, at several
    grid sizes (so workgroup runs end mid-window): bit-exact against the C
    oracle."""
    from gev_amd import _abi
    rng = np.random.default_rng(4242)
    streams = [random_stream(rng, int(rng.integers(1, 40)), max_len=3072) for _ in range(120)]
    empties = b"".join(wo.encode_frame(b"", 2, True, 0, bool(k % 2), b"\x09\x08\x07\x06") for k in range(3000))
    big = bytes(rng.integers(0, 256, 70000, dtype=np.uint8))
    streams.append(wo.encode_frame(big, 2, True, 0, True, b"\x01\x02\x03\x04") + empties +
                   wo.encode_frame(big[:5000], 2, True, 0, True, b"\x05\x06\x07\x08") + empties)
    streams.append(b"".join(wo.encode_frame(bytes(rng.integers(0, 256, int(n), dtype=np.uint8)), 2, True, 0, True,
                                            bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
                            for n in rng.integers(1, 200, 20000)))
    arena, conns = pack_streams(streams)
    i = 0
    try:
        while engine.variant_name(i) is not None:
            engine.set_tuning(_abi.TUNE_UNMASK_VARIANT, i)
            for g in (0, 3, 64):
                engine.set_tuning(_abi.TUNE_UNMASK_GRID, g)
                assert_matches_oracle(engine, arena, conns, f"variant {i} grid {g}")
            i += 1
    finally:
        engine.set_tuning(_abi.TUNE_UNMASK_VARIANT, 0)
        engine.set_tuning(_abi.TUNE_UNMASK_GRID, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c1", "c4", "c5"])
def test_every_unmask_variant_device_synth(engine, cfg):
    """Each unmask variant on a device-generated C1 / C4 / C5-shaped batch:
    decode(mask(P)) == P on every byte via the device verifier."""
    import torch
    import gev_amd
    from gev_amd import _abi, workloads as w
    lay = (w.config_c4(total_payload=192 << 20, n_conns=768, seed=31) if cfg == "c4"
           else w.uniform(8192, 16, 128, opcode=0x1, seed=33) if cfg == "c1"
           else w.config_c5(n_conns=48, messages_per_conn=2, seed=32))
    dev = torch.device("cuda", engine.device)
    arena = torch.zeros(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    desc = torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev)
    conns = torch.from_numpy(lay.conns.copy()).to(dev)
    engine.synth(arena, desc, lay.n_frames, lay.seed)
    out = engine.alloc_batch(lay.n_conns, lay.n_frames, lay.payload_padded)
    i = 0
    try:
        while engine.variant_name(i) is not None:
            engine.set_tuning(_abi.TUNE_UNMASK_VARIANT, i)
            out.payload.fill_(0xAB)
            engine.decode_async(arena, lay.arena_bytes, conns, lay.n_conns, out, lay.n_frames, lay.payload_padded)
            mism = torch.zeros(1, dtype=torch.int64, device=dev)
            engine.verify(desc, lay.n_frames, lay.seed, out, mism)
            torch.cuda.synchronize()
            s = out.summary_host()
            assert int(s["frames"]) == lay.n_frames and int(s["payload_len"]) == lay.payload_len, i
            assert int(mism.item()) == 0, (i, engine.variant_name(i))
            i += 1
    finally:
        engine.set_tuning(_abi.TUNE_UNMASK_VARIANT, 0)


def _uniform_run_streams(rng, n_conns: int):
    """Streams built from runs of equal-size frames (the walk's speculation
    case): run lengths 1-40, frame sizes 2 B-9 KiB, masked/unmasked and long
    length forms that alias to the same frame size, size changes mid-run,
    truncated tails inside a run, and a LEN_MSB header inside a run."""
    streams = []
    for c in range(n_conns):
        s = b""
        for _ in range(int(rng.integers(1, 6))):
            L = int(rng.choice([0, 1, 10, 14, 64, 125, 126, 300, 4096, 9000]))
            masked = bool(rng.random() < 0.8)
            form = None if rng.random() < 0.8 else 64
            for _k in range(int(rng.integers(1, 41))):
                s += wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), 2, True, 0, masked,
                                     bytes(rng.integers(0, 256, 4, dtype=np.uint8)), form)
            if rng.random() < 0.3:  # same frame size, other header: unmasked L+4 vs masked L
                s += wo.encode_frame(bytes(rng.integers(0, 256, L + 4, dtype=np.uint8)), 1, True, 0, False,
                                     b"\0" * 4, form)
        kind = c % 5
        if kind == 1:    # truncated frame of the run's size at the end
            f = wo.encode_frame(bytes(rng.integers(0, 256, 64, dtype=np.uint8)), 2, True, 0, True, b"\1\2\3\4")
            s += b"".join([f] * 9) + f[: int(rng.integers(1, len(f)))]
        elif kind == 2:  # 64-bit length with the MSB set inside a run
            f = wo.encode_frame(b"\x55" * 20, 2, True, 0, True, b"\5\6\7\x08", 64)
            bad = bytearray(f)
            bad[2] |= 0x80
            s += f * 5 + bytes(bad) + f * 3
        streams.append(s)
    return streams


@pytest.mark.gpu
def test_walk_variants_uniform_runs(engine):
    """Both header walks (speculative batches over equal-size runs, and the
    plain chain walk) bit-exact against the C oracle on uniform-run streams,
    on random mixes, and on C2-shaped uniform streams."""
    from gev_amd import _abi
    rng = np.random.default_rng(9090)
    cases = [pack_streams(_uniform_run_streams(rng, 150)),
             pack_streams([random_stream(rng, int(rng.integers(1, 30))) for _ in range(100)]),
             pack_streams([b"".join(wo.encode_frame(bytes(rng.integers(0, 256, 4096, dtype=np.uint8)), 2, True, 0,
                                                    True, bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
                                    for _ in range(n)) for n in (1, 2, 3, 8, 9, 16, 17, 64, 65)])]
    # noise streams (headers parsed from random bytes, MSB-set lengths), long
    # streams of small frames crossing the span walk's LDS ring many times,
    # frames straddling its halves, and an unordered table
    noise = [random_stream(rng, int(rng.integers(0, 4)), max_len=300, tail=False)
             + bytes(rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8)) for _ in range(120)]
    cases.append(pack_streams(noise))
    smalls = [b"".join(wo.encode_frame(bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8)),
                                       int(rng.integers(0, 16)), True, 0, bool(rng.random() < .9),
                                       bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
                       for _ in range(int(rng.integers(200, 900)))) + bytes(int(rng.integers(0, 9)))
              for _ in range(24)]
    smalls += [b"".join(wo.encode_frame(bytes(L), 2, True, 0, True, b"\1\2\3\4") for L in
                        list(range(0, 2100, 7)) + [70000, 3, 5, 1 << 20, 0, 0, 125, 126, 65535, 65536])]
    cases.append(pack_streams(smalls))
    arena, conns = pack_streams([random_stream(rng, int(rng.integers(1, 40))) for _ in range(90)])
    cases.append((arena, conns[rng.permutation(conns.shape[0])]))
    walks = engine.variants(_abi.TUNE_WALK_VARIANT)
    assert walks == [0, 1, 2, 3, 4]
    try:
        for v in walks:
            engine.set_tuning(_abi.TUNE_WALK_VARIANT, v)
            for k, (arena, conns) in enumerate(cases):
                assert_matches_oracle(engine, arena, conns, f"walk variant {v} case {k}")
    finally:
        engine.set_tuning(_abi.TUNE_WALK_VARIANT, 0)


def test_record_pass_groups(engine):
    """The record pass (frames of up to 16 short connections enumerated across
    connection boundaries, long connections one wave each, unrecorded ones
    re-walked) bit-exact on batches of short, long, empty, unrecorded and mixed
    connections, from entries stored by the walking lanes and by the writer
    wave, and with no entries at all."""
    from gev_amd import _abi
    rng = np.random.default_rng(9191)
    cases = []
    for trial in range(3):
        streams = []
        for _ in range(int(rng.integers(50, 700))):
            kind = rng.random()
            if kind < 0.5:    # a few small frames (groups take the enumerated path)
                streams.append(random_stream(rng, int(rng.integers(0, 6)), max_len=200))
            elif kind < 0.7:  # long chains (groups of these go connection by connection)
                streams.append(random_stream(rng, int(rng.integers(60, 200)), max_len=100, tail=False))
            elif kind < 0.8:  # 10-byte frames: more frames than entry slots -> re-walked
                streams.append(b"".join(wo.encode_frame(b"abcd", 1, True, 0, True, b"\1\2\3\4")
                                        for _ in range(int(rng.integers(1, 40)))))
            else:
                streams.append(b"")
        cases.append(pack_streams(streams))
    # exactly 64 x 4 frames in a group, and one more
    for nfr in (16, 17):
        cases.append(pack_streams([b"".join(wo.encode_frame(bytes(20), 2, True, 0, True, b"\1\2\3\4")
                                            for _ in range(nfr)) for _ in range(40)]))
    try:
        for v in (0, 3, 2):
            engine.set_tuning(_abi.TUNE_WALK_VARIANT, v)
            for k, (arena, conns) in enumerate(cases):
                assert_matches_oracle(engine, arena, conns, f"walk variant {v} case {k}")
    finally:
        engine.set_tuning(_abi.TUNE_WALK_VARIANT, 0)


def test_escaped_entry_lengths(engine):
    """The walk's 8-byte entries hold payload lengths below 2^21 - 1; longer
    frames are escaped and the record pass re-reads their header at the
    position its prefix sum gives.  Frames at 2^21 - 2, 2^21 - 1, 2^21 and
    3 MiB, alone, back to back (several escapes in one round of 64 entries),
    first and last on their connection, among small frames, on short
    connections (the grouped pass) and long ones (per connection), through
    the plain and writer walks and the split walk -- bit-exact against the C
    oracle."""
    from gev_amd import _abi
    rng = np.random.default_rng(0xE5C)
    esc = (1 << 21) - 1
    bigs = [esc - 1, esc, esc + 1, 3 << 20]

    def fr(L, form=None):
        return wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), int(rng.choice([1, 2, 0])), True, 0,
                               bool(rng.random() < 0.8), bytes(rng.integers(0, 256, 4, dtype=np.uint8)), form)

    def small(n):
        return b"".join(fr(int(rng.integers(0, 200))) for _ in range(n))

    streams = [
        fr(esc),                                        # alone
        fr(esc - 1) + fr(esc) + fr(esc + 1),            # back to back
        small(3) + fr(3 << 20) + small(2),              # short connection, escape in the middle
        fr(esc + 1) + small(40) + fr(esc) + small(30),  # long connection (> 16 frames)
        small(70) + fr(bigs[int(rng.integers(0, 4))]) + fr(esc) + small(5) + fr(esc, 64)[:-3],  # + cut tail
        small(130) + fr(esc + 7) + small(1),            # escape in the third round of 64
        fr(500, 64) + fr(esc + 2) + fr(esc + 3) + fr(esc + 4) + fr(9),
    ]
    streams += [small(int(rng.integers(0, 20))) + fr(bigs[i % 4]) + small(int(rng.integers(0, 90)))
                for i in range(6)]
    arena, conns = pack_streams(streams)
    knobs = [(_abi.TUNE_WALK_VARIANT, v) for v in (1, 2, 3)]
    knobs += [(_abi.TUNE_SPLIT_LANES, k) for k in (2, 4, 16)]
    defaults = {_abi.TUNE_WALK_VARIANT: 0, _abi.TUNE_SPLIT_LANES: 0}
    try:
        assert_matches_oracle(engine, arena, conns, "default")
        for knob, val in knobs:
            engine.set_tuning(knob, val)
            assert_matches_oracle(engine, arena, conns, f"knob {knob} = {val}")
            engine.set_tuning(knob, defaults[knob])
    finally:
        for knob, val in defaults.items():
            engine.set_tuning(knob, val)


def test_completion_flag_signals_one_launch_passes(engine):
    """gevws_ctx_set_completion_flag: a one-launch decode stores its
    sequence number into the mapped word after its outputs (the host may read
    them once it sees the number, no stream synchronisation); a multi-kernel
    decode reports -1; every one-launch decode takes a new number."""
    import time
    import torch
    arena = gev_amd.PinnedArena(4096)
    rng = np.random.default_rng(4242)
    small = pack_streams([random_stream(rng, 5, max_len=300) for _ in range(40)])
    big = pack_streams([random_stream(rng, 40) for _ in range(60)])
    try:
        engine.set_completion_flag(arena, 64)
        seen = []
        for k in range(3):
            out = gpu_decode(engine, *small)
            seq = engine.completion_seq
            assert seq > 0
            t0 = time.time()
            while int(arena.host[64:68].view(np.uint32)[0]) != seq:
                assert time.time() - t0 < 5, "completion word never written"
            want = ref.decode_batch(np.frombuffer(small[0], np.uint8).copy(), small[1][:, 0], small[1][:, 1])
            assert out.frames_host().tobytes() == want["frames"].tobytes()
            seen.append(seq)
        assert seen == sorted(set(seen))
        gpu_decode(engine, *big)
        assert engine.completion_seq == -1  # > 128 KiB: the multi-kernel decode
        torch.cuda.synchronize()
    finally:
        engine.set_completion_flag(None)
        torch.cuda.synchronize()
        arena.close()
    assert engine.completion_seq == -1


def test_walk_variant_knob_bounds(engine):
    from gev_amd import _abi
    with pytest.raises(ValueError):
        engine.set_tuning(_abi.TUNE_WALK_VARIANT, len(engine.variants(_abi.TUNE_WALK_VARIANT)))
    with pytest.raises(ValueError):
        engine.set_tuning(_abi.TUNE_WALK_VARIANT, -1)
    with pytest.raises(ValueError):
        engine.set_tuning(_abi.TUNE_UNMASK_VARIANT, len(engine.variants(_abi.TUNE_UNMASK_VARIANT)))
    for key in _abi.TUNE_RETIRED:  # round 1-3 measurement knobs are gone
        with pytest.raises(ValueError):
            engine.set_tuning(key, 0)


@pytest.mark.gpu
def test_copy_helper_copies_and_rejects_unknown_flags(engine):
    """gevws_copy_async (the bench's copy ceiling): every load / layout flag
    copies the bytes exactly, from an aligned and a misaligned source; an
    unknown flag bit is GEVWS_ERR_INVALID, not silently masked (ABI 2,
    ADVICE r4)."""
    import torch
    dev = torch.device("cuda", engine.device)
    n = 3 * 4096 * 16 + 4096 + 48  # whole tiles per workgroup, a partial step and a tail
    src = torch.randint(0, 256, (n + 64,), dtype=torch.uint8, device=dev)
    for flags in (0, 0x40000000, 0x20000000, 0x20000000 | 0x40000000, 0x10000000, 0x08000000):
        for so in (0, 7):
            dst = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
            engine.copy_(dst, src, n, src_offset=so, grid=flags | 3)
            torch.cuda.synchronize()
            assert torch.equal(dst[:n], src[so:so + n]), (hex(flags), so)
            assert int(dst[n:].sum()) == 0
    with pytest.raises(RuntimeError):
        engine.copy_(dst, src, n, grid=0x80000000)


@pytest.mark.gpu
@pytest.mark.parametrize("L", [3001, 128])
def test_v3_counter_runs_equal_frames_across_tiles(engine, L):
    """The v3 path's counter runs: equal-size frames that do not
    line up with tiles (3001 B: every source alignment in turn; 128 B + 8-byte
    headers) in batches of > 512 / 768 tiles, decoded with 8 and 12
    workgroups (GEVWS_TUNE_UNMASK_GRID turns off the big-frame grid, so
    every workgroup takes 16-tile runs from the per-XCD counters), for the
    default and the round-4 variant: bit-exact against the C oracle."""
    from gev_amd import _abi
    rng = np.random.default_rng(L)
    n = 1100 if L == 3001 else 25000
    per = n // 40
    streams = [b"".join(wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), 2, True, 0, True,
                                        bytes(rng.integers(0, 256, 4, dtype=np.uint8))) for _ in range(per))
               for _ in range(40)]
    arena, conns = pack_streams(streams)
    assert (L + 15) // 16 * 16 * per * 40 // 4096 >= 768
    try:
        for v in (0, 2):
            engine.set_tuning(_abi.TUNE_UNMASK_VARIANT, v)
            for g in (8, 12):
                engine.set_tuning(_abi.TUNE_UNMASK_GRID, g)
                got = assert_matches_oracle(engine, arena, conns, f"L {L} variant {v} grid {g}")
                assert int(got["summary"]["run_frames"]) * 2 >= got["frames"].shape[0]  # the v3 path ran
    finally:
        engine.set_tuning(_abi.TUNE_UNMASK_VARIANT, 0)
        engine.set_tuning(_abi.TUNE_UNMASK_GRID, 0)


def _frames_of_exactly(rng, nbytes: int) -> bytes:
    """Masked frames of random sizes whose wire bytes add up to exactly nbytes (0 or >= 6)."""
    out = b""
    while nbytes:
        assert nbytes >= 6
        if nbytes <= 131:                      # one 6-byte-header frame closes it
            L = nbytes - 6
        elif nbytes < 140:                     # a 66-byte frame, then one that closes it
            L = 60
        else:
            L = int(rng.integers(0, min(1200, nbytes - 140) + 1))
        f = wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), int(rng.choice([0, 1, 2, 9, 10])),
                            True, 0, True, bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
        out += f
        nbytes -= len(f)
    return out


@pytest.mark.gpu
def test_one_launch_decode_at_its_limits(engine):
    """The one-launch decode stages its whole input in LDS, in two shapes
    (round 6): 256 lanes / 64 KiB and 1 024 lanes / 128 KiB.  At each shape's
    limits -- N connections ending on the last byte of exactly B bytes, the
    last one with a cut frame; one connection of frames and a 5-byte tail;
    N - 1 empty connections beside one payload frame filling B; a 6-byte frame
    whose header starts 6 bytes before the end -- and just past the narrow
    shape's (257 connections; 65 537 bytes): bit-exact against the C oracle in
    one launch and in the multi-kernel path; the one launch also with a
    completion flag set, which stages the input through up to 32 workgroups'
    tagged slices (a live pass's form).  A batch past the wide shape (1 025
    connections; 131 073 bytes) takes the multi-kernel path."""
    import torch
    from gev_amd import _abi
    rng = np.random.default_rng(65536)

    def at_limits(n_conns, nbytes, max_len):
        cases = []
        streams = [random_stream(rng, int(rng.integers(0, 3)), max_len=max_len, tail=False)
                   for _ in range(n_conns - 1)]
        last = nbytes - sum(len(s) for s in streams)
        assert last > 300
        streams.append(_frames_of_exactly(rng, last + 300)[:last])  # cut inside a frame
        cases.append(pack_streams(streams))
        cases.append(pack_streams([_frames_of_exactly(rng, nbytes - 5) + b"\x82\x85\x01\x02\x03"]))
        L = nbytes - (8 if nbytes - 8 <= 0xFFFF else 14)
        big = wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), 2, True, 0, True, b"\x0a\x0b\x0c\x0d")
        assert len(big) == nbytes
        cases.append(pack_streams([b""] * (n_conns - 1) + [big]))
        cases.append(pack_streams([_frames_of_exactly(rng, nbytes - 6) + wo.encode_frame(b"", 9, True, 0, True,
                                                                                          b"\1\2\3\4")]))
        return cases

    narrow = at_limits(256, 65536, 200)
    wide = at_limits(1024, 131072, 100)
    past_narrow = [pack_streams([random_stream(rng, 1, max_len=120, tail=False) for _ in range(257)]),
                   pack_streams([_frames_of_exactly(rng, 65537)])]
    past_wide = [pack_streams([random_stream(rng, 1, max_len=60, tail=False) for _ in range(1025)]),
                 pack_streams([_frames_of_exactly(rng, 131073)])]
    for arena, conns in narrow:
        assert len(arena) == 65536 and conns.shape[0] <= 256
    for arena, conns in wide:
        assert len(arena) == 131072 and conns.shape[0] <= 1024
    assert past_wide[0][1].shape[0] == 1025 and len(past_wide[1][0]) == 131073
    flag = gev_amd.PinnedArena(4096)
    try:
        for sb, flagged in ((_abi.ONE_LAUNCH_MAX_BYTES, False), (_abi.ONE_LAUNCH_MAX_BYTES, True), (0, False)):
            engine.set_tuning(_abi.TUNE_SMALL_BATCH, sb)
            engine.set_completion_flag(flag if flagged else None, 64)
            for k, (arena, conns) in enumerate(narrow + wide + past_narrow + past_wide):
                assert_matches_oracle(engine, arena, conns, f"case {k} small_batch {sb} flagged {flagged}")
                if flagged:
                    one = k < len(narrow + wide + past_narrow)
                    assert (engine.completion_seq > 0) == one, k
    finally:
        engine.set_tuning(_abi.TUNE_SMALL_BATCH, _abi.ONE_LAUNCH_MAX_BYTES)
        engine.set_completion_flag(None)
        torch.cuda.synchronize()
        flag.close()
