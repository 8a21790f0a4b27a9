"""GPU parity for the outbound encode: the device
ws.WriteHeader (write.go:48-84) + ws.FrameToBytes (frame.go:274-278), through
the C ABI (gevws_encode_batch_async), bit-exact against the golden vectors and
the C oracle, plus the echo round trip decode -> NewBinaryFrame reply ->
encode -> decode (benchmarks/websocket/server.go:22-29)."""
import numpy as np
import pytest

import gev_amd
from oracle import ref
from oracle import ws_oracle as wo
from tests._helpers import gpu_decode, host_result, pack_streams, random_stream

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[0, 1, 2, 3, 4, 5],
                ids=["auto", "one_tile", "two_tiles", "two_tiles_contiguous", "two_tiles_cyclic", "two_tiles_counter"])
def enc_variant(request, engine):
    """Every form of the encode kernel k_encode6 (GEVWS_TUNE_ENCODE_VARIANT):
    0 = the default (its step and run mode chosen per batch), 1 / 2 = one /
    two tiles a wave step, 3 / 4 / 5 = two tiles a step with contiguous /
    cyclic / counter runs."""
    try:
        engine.set_tuning(gev_amd._abi.TUNE_ENCODE_VARIANT, request.param)
    except RuntimeError:
        pytest.skip("no such encode variant")
    yield request.param
    engine.set_tuning(gev_amd._abi.TUNE_ENCODE_VARIANT, 0)


def _dev(engine):
    import torch
    return torch.device("cuda", engine.device)


def _records(hdrs16: np.ndarray, offs, lens) -> np.ndarray:
    fr = np.zeros(hdrs16.shape[0], gev_amd.OUT_FRAME_DTYPE)
    fr.view(np.uint8).reshape(-1, 32)[:, :16] = hdrs16
    fr["payload_off"] = offs
    fr["payload_len"] = lens
    return fr


def _encode_check(engine, fr: np.ndarray, payload: np.ndarray, tag=""):
    import torch
    d_pay = torch.from_numpy(np.concatenate([payload, np.zeros(16, np.uint8)])).to(_dev(engine))
    wire, off = engine.encode(fr, d_pay)
    want, woff = ref.encode_batch(fr, payload)
    got = wire.cpu().numpy()
    assert got.size == want.size, tag
    assert np.array_equal(got, want), (tag, int(np.argmax(got != want)))
    assert np.array_equal(off, woff), tag
    return got


def test_encode_golden(engine, golden, enc_variant):
    g = golden["encode"]
    offs = np.concatenate([[0], np.cumsum(g["payload_len"])[:-1]]).astype(np.uint64)
    fr = _records(g["hdr"], offs, g["payload_len"])
    got = _encode_check(engine, fr, g["payload"], "golden")
    assert np.array_equal(got, g["wire"])


def test_encode_random_and_tiny_frames(engine, enc_variant):
    """Random batches: payloads out of frame order, every header form, RSV /
    opcode bytes outside the spec, lengths that disagree with the payload
    (Go's byte arithmetic), 1 to 5 000 frames, up to 200 KB each: aligned-load
    streaming inside payloads, frame windows queueing every 64-byte group that
    holds a frame boundary for the workgroup's assembly pass."""
    _encode_random(engine)


def test_encode_capacity_error_leaves_wire_sizes(engine, enc_variant):
    """A wire total past out_cap: GEVWS_ERR_CAPACITY, the summary still holds
    the totals, and d_out_off[f] holds frame f's wire size h + L (the contract
    of include/gevws.h) -- 20 000 frames over several offset-pass
    workgroups.  The exact capacity then encodes."""
    import torch
    rng = np.random.default_rng(77)
    n = 20000
    lens = rng.integers(0, 400, n)
    lens[rng.integers(0, n, 20)] = rng.integers(126, 70000, 20)  # 4- and 10-byte headers too
    payload = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    hd = np.array([np.frombuffer(wo.Header(True, 0, 2, bool(i % 3 == 0), b"\1\2\3\4", int(L)).pack(), np.uint8)
                   for i, L in enumerate(lens)])
    fr = _records(hd, offs, lens)
    want, woff = ref.encode_batch(fr, payload)
    total = int(want.size)
    sizes = np.diff(np.append(woff, np.uint64(total)))
    dev = _dev(engine)
    d_fr = torch.from_numpy(fr.view(np.uint8).reshape(-1, 32).copy()).to(dev)
    d_pay = torch.from_numpy(np.concatenate([payload, np.zeros(16, np.uint8)])).to(dev)
    wire = torch.zeros(total + gev_amd._abi.OUT_PAD, dtype=torch.uint8, device=dev)
    off = torch.zeros(n, dtype=torch.int64, device=dev)
    summ = torch.zeros(64, dtype=torch.uint8, device=dev)
    for cap in (total - 1, total // 2, 0):
        engine.encode_async(d_fr, n, d_pay, wire, cap, off, summ)
        torch.cuda.synchronize(dev)
        s = summ.cpu().numpy().view(gev_amd.SUMMARY_DTYPE)[0]
        assert int(s["status"]) == gev_amd.ERR_CAPACITY, cap
        assert int(s["frames"]) == n and int(s["payload_bytes"]) == total, cap
        assert int(s["payload_len"]) == int(lens.sum()), cap
        assert np.array_equal(off.cpu().numpy().astype(np.uint64), sizes), cap
    engine.encode_async(d_fr, n, d_pay, wire, total, off, summ)
    torch.cuda.synchronize(dev)
    s = summ.cpu().numpy().view(gev_amd.SUMMARY_DTYPE)[0]
    assert int(s["status"]) == 0 and int(s["payload_bytes"]) == total
    assert np.array_equal(off.cpu().numpy().astype(np.uint64), woff)
    assert np.array_equal(wire[:total].cpu().numpy(), want)


def _encode_random(engine):
    rng = np.random.default_rng(41)
    # (4000, 120) / (2500, 250): 64-128 frames in a two-tile step, the second
    # round of k_encode6's frame-offset scan
    for trial, (n, maxlen) in enumerate([(1, 0), (5, 10), (300, 3000), (3000, 0), (5000, 20), (200, 70000),
                                         (60, 200000), (4000, 120), (2500, 250)]):
        lens = rng.integers(0, maxlen + 1, n)
        payload = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        perm = rng.permutation(n)           # payloads need not be in frame order
        hd = []
        for i in range(n):
            h = wo.Header(bool(rng.random() < .7), int(rng.integers(0, 256)) if rng.random() < .1 else 0,
                          int(rng.integers(0, 16)), bool(rng.random() < .3),
                          bytes(rng.integers(0, 256, 4, dtype=np.uint8)),
                          int(lens[perm[i]]) if rng.random() < .9 else int(rng.integers(-5, 70000)))
            hd.append(np.frombuffer(h.pack(), np.uint8))
        fr = _records(np.array(hd), offs[perm], lens[perm])
        _encode_check(engine, fr, payload, f"trial {trial}")


def _uniform_frames(wire_len: int, n: int, rng):
    """n unmasked binary frames of `wire_len` wire bytes each (2-byte header)."""
    L = wire_len - 2
    payload = rng.integers(0, 256, n * L + 1, dtype=np.uint8)
    hd = np.array([np.frombuffer(wo.Header(True, 0, 2, False, b"\0\0\0\0", L).pack(), np.uint8)
                   for _ in range(n)])
    offs = (np.arange(n, dtype=np.uint64) * np.uint64(L))
    return _records(hd, offs, np.full(n, L)), payload


def test_encode_window_queue_at_capacity(engine, enc_variant):
    """Windows whose boundary queues are as full as they get: 1 024 frames
    of 16 wire bytes in one 4-tile window (every chunk holds a header, so the
    workgroup queue takes all 1 024 chunks -- as single chunks or as 256
    whole 64-byte groups -- and F = the window's frame capacity); one frame
    more (the per-lane fallback); frames of 32 B (every other 64-byte group
    half header); frames of 17 / 24 / 33 B (boundaries at every phase, groups
    with one to four boundaries); and runs of tiny frames between big ones
    (three or more frames per chunk).  Regression test for the queue's
    capacity and for groups cut by the batch's end (sentinel slots)."""
    rng = np.random.default_rng(1234)
    for wl, n in [(16, 1024), (16, 1025), (32, 512), (32, 513), (17, 963), (24, 682), (33, 1000),
                  (16, 1024 * 3), (32, 512 * 5),
                  # 33 / 40 / 64 B put a boundary in every 64-byte group (a step's whole queue)
                  (32, 1024), (32, 1025), (33, 2000), (40, 1700), (64, 1100), (16, 2048 * 2),
                  # k_encode6's step tables (64 frames a tile, 128 a two-tile step): 64-66 B
                  # frames put 63-65 frames in a tile, 70 B about 118 in a step
                  (64, 2000), (65, 2000), (66, 2000), (70, 3000)]:
        fr, pay = _uniform_frames(wl, n, rng)
        _encode_check(engine, fr, pay, f"{wl}B x {n}")
    lens = np.concatenate([rng.integers(0, 4, 200), [20000], rng.integers(0, 14, 700), [9000],
                           rng.integers(0, 40, 400)])
    payload = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    hd = np.array([np.frombuffer(wo.Header(True, 0, 2, False, b"\0\0\0\0", int(L)).pack(), np.uint8)
                   for L in lens])
    _encode_check(engine, _records(hd, offs, lens), payload, "tiny runs")


def _arena_batch(rng, lens, p0=0, hdr_len=None):
    """Replies whose payloads sit in a decode's payload-arena layout: slots of
    round16(L) bytes back to back from a 16-aligned p0 (an echo server's case)."""
    lens = np.asarray(lens, dtype=np.int64)
    slots = (lens + 15) // 16 * 16
    offs = p0 + np.concatenate([[0], np.cumsum(slots)[:-1]]).astype(np.uint64)
    payload = rng.integers(0, 256, int(p0 + slots.sum()) + 16, dtype=np.uint8)
    hd = []
    for i, L in enumerate(lens):
        hl = int(L) if hdr_len is None else hdr_len(i, int(L))
        h = wo.Header(bool(rng.random() < .8), 0, int(rng.choice([1, 2, 9, 10])), bool(rng.random() < .3),
                      bytes(rng.integers(0, 256, 4, dtype=np.uint8)), hl)
        hd.append(np.frombuffer(h.pack(), np.uint8))
    return _records(np.array(hd), offs, lens), payload


def test_encode_decode_arena_layouts(engine, enc_variant):
    """Payload slots back to back as a decode leaves them (an echo server's
    replies) -- every header form, empty frames first / last / in runs longer
    than a window's table, 1-15 byte tails, frames spanning many streaming
    steps, a batch of only empty frames, and a p0 past the arena start; plus
    one slot out of place."""
    rng = np.random.default_rng(77)
    cases = [
        [0, 5, 0, 130, 1, 15, 16, 17, 0],
        list(rng.integers(0, 300, 3000)),
        list(rng.integers(64, 4096, 2000)),
        [0] * 1500 + [100] + [0] * 1300 + [3],
        [0, 0, 0],
        [70000, 1, 300000, 0, 65536, 65535, 131072 + 7],
        list(np.clip((64 * (1 - rng.random(20000)) ** (-1 / 1.1)).astype(np.int64), 64, 1 << 20)),
    ]
    for k, lens in enumerate(cases):
        fr, pay = _arena_batch(rng, lens, p0=16 * int(rng.integers(0, 5)))
        _encode_check(engine, fr, pay, f"arena case {k}")
    # one slot moved: not the arena layout
    fr, pay = _arena_batch(rng, list(rng.integers(0, 500, 200)))
    fr["payload_off"][57] += 16
    _encode_check(engine, fr, pay, "arena layout broken")
    # header lengths that disagree with the payload (Go's byte arithmetic)
    fr, pay = _arena_batch(rng, list(rng.integers(0, 500, 300)), hdr_len=lambda i, L: (L * 7 + i) % 70000)
    _encode_check(engine, fr, pay, "arena, odd header lengths")


def test_encode_empty_batch(engine):
    import torch
    fr = np.zeros(0, gev_amd.OUT_FRAME_DTYPE)
    wire, off = engine.encode(fr, torch.zeros(16, dtype=torch.uint8, device=_dev(engine)))
    assert wire.numel() == 0 and off.size == 0


def test_echo_round_trip_on_device(engine, enc_variant):
    """Client frames (masked) -> device decode -> server replies
    NewBinaryFrame(payload) whose payloads are the decoded arena slots -> device
    encode -> device decode of the reply stream: the same payload bytes."""
    import torch
    rng = np.random.default_rng(42)
    streams = [random_stream(rng, int(rng.integers(0, 30)), max_len=5000) for _ in range(40)]
    arena, conns = pack_streams(streams)
    out = gpu_decode(engine, arena, conns)
    got = host_result(out)
    f = got["frames"]
    n = f.shape[0]
    replies = np.zeros(n, gev_amd.OUT_FRAME_DTYPE)
    replies["fin"] = 1
    replies["opcode"] = wo.OP_BINARY
    replies["length"] = f["length"]
    replies["payload_off"] = f["payload_off"]
    replies["payload_len"] = f["length"]
    wire, off = engine.encode(replies, out.payload)
    w = wire.cpu().numpy()
    # the oracle builds the same reply bytes from the oracle's own decode
    want = b"".join(wo.frame_to_bytes(*wo.new_frame(wo.OP_BINARY, True,
                                                   got["payload"][int(o):int(o) + int(L)].tobytes()))
                    for o, L in zip(f["payload_off"], f["length"]))
    assert w.tobytes() == want
    # trail with 5 bytes of an incomplete 127-form header: avail >= 6 for every
    # real frame (read.go:20-23) without adding a decodable frame
    tail = np.array([0x82, 0x7F, 0, 0, 0], np.uint8)
    back = host_result(gpu_decode(engine, np.concatenate([w, tail]), np.array([[0, w.size + 5]])))
    assert int(back["summary"]["frames"]) == n
    assert np.array_equal(back["payload"], got["payload"])  # same 16-byte-aligned arena layout


def test_echo_round_trip_c2_full_size(engine, enc_variant):
    """Full C2 batch (262 144 x 4 KiB): decode, encode the binary replies,
    decode the reply stream, compare the payload arenas on the device."""
    import torch
    from gev_amd import workloads
    lay = workloads.config_c2()
    dev = _dev(engine)
    arena = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    arena[lay.arena_bytes:] = 0
    engine.synth(arena, torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev), lay.n_frames, lay.seed)
    conns = torch.from_numpy(lay.conns.copy()).to(dev)
    out = engine.decode(arena, lay.arena_bytes, conns, lay.n_conns, lay.n_frames, lay.payload_padded)
    f = out.frames[: lay.n_frames].cpu().numpy().reshape(-1).view(gev_amd.FRAME_DTYPE)
    replies = np.zeros(lay.n_frames, gev_amd.OUT_FRAME_DTYPE)
    replies["fin"], replies["opcode"] = 1, wo.OP_BINARY
    replies["length"] = f["length"]
    replies["payload_off"], replies["payload_len"] = f["payload_off"], f["length"]
    wire, _ = engine.encode(replies, out.payload)
    assert wire.numel() == lay.n_frames * (4 + 4096)
    w2 = torch.zeros(wire.numel() + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    w2[: wire.numel()] = wire   # 4 KiB frames: every frame already has >= 6 bytes behind it
    c2 = torch.tensor([[0, wire.numel()]], dtype=torch.int64, device=dev)
    back = engine.decode(w2, wire.numel(), c2, 1, lay.n_frames, lay.payload_padded)
    assert int(back.summary_host()["frames"]) == lay.n_frames
    assert torch.equal(back.payload[: lay.payload_padded], out.payload[: lay.payload_padded])
