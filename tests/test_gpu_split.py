"""Split header walk (k_walk_split, GEVWS_TUNE_SPLIT_LANES): lanes guess frame
starts inside long streams and walk the segments between guesses; a
connection is accepted only when every segment ends exactly on the next
guess, else it is re-walked serially.  Whatever the guesses, the output must
be the serial chain's: every case below is compared with the oracle
(oracle/ws_ref.c) record by record, byte by byte, per connection and in the
summary (run_frames included), for every lane count and the auto choice.

The cases aim at each way a guess can go: small frames (guesses confirmed),
big frames (no header near a split point), a payload that carries a
plausible embedded frame chain (a confirmed guess that is NOT a frame start),
noise, an ERR_LEN_MSB header mid-stream, 2-5 byte frames (the avail < 6
rule at a segment's end), uniform frames (run_frames stitched across
segments), partial tails, unordered tables and streams outside the arena."""
import numpy as np
import pytest

from oracle import ref
from oracle import ws_oracle as wo
from tests._helpers import assert_matches_oracle, gpu_decode, host_result, pack_streams

pytestmark = pytest.mark.gpu

KEY = b"\x11\x22\x33\x44"


def _frames(rng, nbytes, lens, masked=True, opcode=2):
    """Frames with payload lengths drawn by lens(rng) until nbytes of stream."""
    out, tot = [], 0
    while tot < nbytes:
        L = int(lens(rng))
        f = wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), opcode, True, 0, masked,
                            bytes(rng.integers(0, 256, 4, dtype=np.uint8)) if masked else KEY)
        out.append(f)
        tot += len(f)
    return b"".join(out)


def _power(rng):
    u = rng.random()
    return min(int(64 * (1 - u * (1 - (64 / (1 << 20)) ** 1.1)) ** (-1 / 1.1)), 1 << 20)


def _tail(rng):
    t = wo.encode_frame(bytes(300), 2, True, 0, True, KEY)
    return t[: int(rng.integers(1, len(t)))]


def _cases():
    rng = np.random.default_rng(0x5911)
    cases = {}
    # long chains of small frames, some with a partial last frame
    small = [_frames(rng, int(rng.integers(40_000, 300_000)), lambda r: r.integers(0, 200))
             + (_tail(rng) if k % 3 == 0 else b"") for k in range(48)]
    cases["small"] = pack_streams(small)
    # power-law frames 64 B .. 1 MiB (C4's mix)
    cases["power"] = pack_streams([_frames(rng, int(rng.integers(100_000, 1_500_000)), _power) for _ in range(24)])
    # an unmasked first frame whose payload is itself a plausible stream of
    # unmasked frames: split points inside it confirm guesses that are not
    # frame starts
    fake = []
    for k in range(12):
        inner = _frames(rng, int(rng.integers(60_000, 120_000)), lambda r: r.integers(0, 120), masked=False)
        outer = wo.encode_frame(inner, 2, True, 0, False, KEY)
        fake.append(outer + _frames(rng, int(rng.integers(0, 80_000)), lambda r: r.integers(0, 120), masked=False))
    cases["embedded_chain"] = pack_streams(fake)
    # noise: headers parsed from random bytes
    cases["noise"] = pack_streams([bytes(rng.integers(0, 256, int(rng.integers(33_000, 200_000)), dtype=np.uint8))
                                   for _ in range(16)])
    # ERR_LEN_MSB header in the middle of a long small-frame chain
    msb = bytes([0x82, 0xFF, 0x80, 0, 0, 0, 0, 0, 0, 5, 1, 2, 3, 4]) + b"hello"
    errs = []
    for _ in range(8):
        a = _frames(rng, int(rng.integers(30_000, 150_000)), lambda r: r.integers(0, 150))
        b = _frames(rng, int(rng.integers(30_000, 150_000)), lambda r: r.integers(0, 150))
        errs.append(a + msb + b)
    cases["len_msb"] = pack_streams(errs)
    # 2..5-byte unmasked frames: a segment's last frames meet avail < 6
    tiny = [_frames(rng, int(rng.integers(33_000, 90_000)), lambda r: r.integers(0, 4), masked=False)
            for _ in range(10)]
    cases["tiny"] = pack_streams(tiny)
    # uniform frames (run_frames counts pairs across segment boundaries)
    cases["uniform"] = pack_streams([_frames(rng, 200_000, lambda r: 100) for _ in range(20)]
                                    + [_frames(rng, 300_000, lambda r: 4096) for _ in range(8)])
    # mixed: short and empty connections between long ones
    mixed = []
    for k in range(60):
        if k % 4 == 0:
            mixed.append(b"")
        elif k % 4 == 1:
            mixed.append(_frames(rng, int(rng.integers(1, 3000)), lambda r: r.integers(0, 300)))
        else:
            mixed.append(_frames(rng, int(rng.integers(32_768, 250_000)), lambda r: r.integers(0, 500)))
    cases["mixed"] = pack_streams(mixed)
    arena, conns = cases["small"]
    cases["unordered"] = (arena, conns[rng.permutation(conns.shape[0])])
    return cases


@pytest.fixture(scope="module")
def split_cases():
    return _cases()


@pytest.mark.parametrize("lanes,min_seg,wv", [(0, 16384, 0), (2, 16384, 0), (4, 16384, 0), (8, 16384, 0),
                                              (16, 16384, 0), (32, 16384, 0), (32, 4096, 0), (16, 1024, 0),
                                              (16, 16384, 4), (2, 1024, 4)])
def test_split_walk_matches_oracle(engine, split_cases, lanes, min_seg, wv):
    """Every lane count (32: two connections per wave), and shorter minimum
    segments (GEVWS_TUNE_SPLIT_MIN_BYTES: more guesses per connection, each
    nearer the previous one); entries through the writer wave (the default)
    and from the walking lanes (walk variant 4)."""
    from gev_amd import _abi
    engine.set_tuning(_abi.TUNE_SMALL_BATCH, 0)
    engine.set_tuning(_abi.TUNE_SPLIT_LANES, lanes)
    engine.set_tuning(_abi.TUNE_SPLIT_MIN_BYTES, min_seg)
    engine.set_tuning(_abi.TUNE_WALK_VARIANT, wv)
    try:
        for name, (arena, conns) in split_cases.items():
            assert_matches_oracle(engine, arena, conns, f"split lanes {lanes} min {min_seg} walk {wv}: {name}")
    finally:
        engine.set_tuning(_abi.TUNE_WALK_VARIANT, 0)
        engine.set_tuning(_abi.TUNE_SPLIT_LANES, 0)
        engine.set_tuning(_abi.TUNE_SPLIT_MIN_BYTES, 16384)
        engine.set_tuning(_abi.TUNE_SMALL_BATCH, _abi.ONE_LAUNCH_MAX_BYTES)


def test_split_walk_streams_outside_the_arena(engine, split_cases):
    """Out-of-arena rows in a split batch: GEVWS_ERR_INVALID, nothing read,
    the long connections around them exact."""
    import gev_amd
    from gev_amd import _abi
    arena, conns = split_cases["small"]
    n = len(arena)
    bad = np.array([[n - 4, 10], [n + 100, 70_000], [1 << 62, 1 << 62]], np.int64)
    table = np.concatenate([conns[:3], bad[:1], conns[3:5], bad[1:], conns[5:]])
    engine.set_tuning(_abi.TUNE_SPLIT_LANES, 8)
    try:
        got = host_result(gpu_decode(engine, arena, table))
    finally:
        engine.set_tuning(_abi.TUNE_SPLIT_LANES, 0)
    st = got["conn_out"]["status"]
    assert list(st[[3, 6, 7]]) == [gev_amd.ERR_INVALID] * 3
    assert int(got["summary"]["errors"]) == 3
    want = ref.decode_batch(np.frombuffer(arena, np.uint8).copy(), conns[:, 0], conns[:, 1])
    assert got["frames"].tobytes() == want["frames"].tobytes()
    assert np.array_equal(got["payload"], want["payload"])


def test_split_lanes_knob_bounds(engine):
    from gev_amd import _abi
    for bad in (-1, 3, 6, 64):
        with pytest.raises(ValueError):
            engine.set_tuning(_abi.TUNE_SPLIT_LANES, bad)
    engine.set_tuning(_abi.TUNE_SPLIT_LANES, 0)
    for knob, bad in ((_abi.TUNE_SPLIT_MIN_BYTES, 1023), (_abi.TUNE_SPLIT_LANES_PER_CU, 63)):
        with pytest.raises(ValueError):
            engine.set_tuning(knob, bad)


def test_split_walk_auto_choice(engine, split_cases):
    """Auto (GEVWS_TUNE_SPLIT_LANES 0): a context splits a batch of few long
    connections once a finished decode on it showed long chains of small
    frames -- not on its first batch, not after big frames -- and the split
    decode is exact."""
    import torch
    from gev_amd import _abi
    rng = np.random.default_rng(77)
    longs = pack_streams([_frames(rng, 300_000, lambda r: r.integers(0, 200)) for _ in range(64)])
    bigs = pack_streams([_frames(rng, 300_000, lambda r: 8192) for _ in range(64)])
    engine.set_tuning(_abi.TUNE_SMALL_BATCH, 0)
    try:
        assert_matches_oracle(engine, *bigs, "auto: big frames")
        torch.cuda.synchronize()
        assert_matches_oracle(engine, *longs, "auto: after big frames")
        assert engine.last_split_lanes == 1
        torch.cuda.synchronize()
        assert_matches_oracle(engine, *longs, "auto: after long chains")
        assert engine.last_split_lanes == 16
        torch.cuda.synchronize()
        assert_matches_oracle(engine, *bigs, "auto: big frames after long chains")
        assert engine.last_split_lanes == 16  # the previous batch decides
        torch.cuda.synchronize()
        assert_matches_oracle(engine, *bigs, "auto: big frames again")
        assert engine.last_split_lanes == 1
    finally:
        engine.set_tuning(_abi.TUNE_SMALL_BATCH, _abi.ONE_LAUNCH_MAX_BYTES)


def test_wide_unmask_grid_after_mixed_batch(engine):
    """The unmask's wide grid (32 workgroups per CU) is launched after a
    finished decode of a mixed-size batch below 8 GiB of output, and the
    kernel uses it only when this batch is mixed as well: both cases exact
    (every byte by the generator property, leading connections against the
    oracle)."""
    import torch
    from gev_amd import workloads as w
    from tests.test_gpu_parity import _synth_decode_verify
    mixed = w.config_c4(total_payload=512 << 20, n_conns=1024, seed=5)       # 131 K output tiles, v5
    uniform = w.uniform(1024, 128, 4096, seed=6)                             # 512 MiB of 4 KiB frames, v3
    ncu = torch.cuda.get_device_properties(engine.device).multi_processor_count
    _synth_decode_verify(engine, uniform, check_slice_conns=4)
    _synth_decode_verify(engine, mixed, check_slice_conns=4)
    assert engine.last_unmask_grid <= 4 * ncu
    _synth_decode_verify(engine, mixed, check_slice_conns=4)   # after a mixed batch: wide grid, used
    assert engine.last_unmask_grid > 4 * ncu, engine.last_unmask_grid
    _synth_decode_verify(engine, uniform, check_slice_conns=4)  # wide launch, the usual grid used
    assert engine.last_unmask_grid > 4 * ncu
    _synth_decode_verify(engine, uniform, check_slice_conns=4)
    assert engine.last_unmask_grid <= 4 * ncu


def test_split_walk_counts_its_serial_rewalks(engine, split_cases):
    """gevws_ctx_last_split_fallbacks: the connections whose guesses did not
    line up and were re-walked serially.  A payload carrying a plausible
    embedded chain makes guesses that are not frame starts (every such
    connection re-walked), chains of small frames are accepted as guessed
    (none), an unsplit decode reports 0 -- and the output is the oracle's
    every time."""
    from gev_amd import _abi
    engine.set_tuning(_abi.TUNE_SMALL_BATCH, 0)
    engine.set_tuning(_abi.TUNE_SPLIT_LANES, 16)
    try:
        counts = {}
        for name in ("embedded_chain", "small", "power"):
            arena, conns = split_cases[name]
            assert_matches_oracle(engine, arena, conns, f"fallbacks: {name}")
            assert engine.last_split_lanes == 16
            counts[name] = engine.last_split_fallbacks
            assert 0 <= counts[name] <= conns.shape[0], (name, counts[name])
        assert counts["embedded_chain"] > 0, counts
        assert counts["small"] == 0, counts
        engine.set_tuning(_abi.TUNE_SPLIT_LANES, 1)
        assert_matches_oracle(engine, *split_cases["embedded_chain"], "fallbacks: unsplit")
        assert engine.last_split_lanes == 1 and engine.last_split_fallbacks == 0
    finally:
        engine.set_tuning(_abi.TUNE_SPLIT_LANES, 0)
        engine.set_tuning(_abi.TUNE_SMALL_BATCH, _abi.ONE_LAUNCH_MAX_BYTES)
