"""Property-based parity on the device (hypothesis, shrinking to a minimal
failing batch): the HIP decode equals the C oracle (oracle/ws_ref.c, the
restatement of read.go:19-84 + protocol.go:38-62 + connection.go:208-218)
bit-exactly on generated batches -- every length class, minimal and
non-minimal length forms, any RSV / opcode, masked and unmasked frames,
garbage tails -- through the one-launch path and, with it turned off
(GEVWS_TUNE_SMALL_BATCH = 0), the multi-kernel path; and the device
ws.Cipher (cipher.go:14-53) equals the bytewise one at any offset and
alignment; the device encode (FrameToBytes) equals the C oracle's on
generated records; the device handler step (dispatch + encode of the
replies) equals oracle/ws_oracle.on_message on generated control-heavy
streams; the host Protocol over ring buffers fed in arbitrary chunks hands
every connection the oracle's frames and keeps its incomplete tail; the
split header walk equals the serial chain on generated long streams with
adversarial content (embedded frame chains, noise, tiny frames); the
unmask's paths (v3 windows, counter runs, v5) over >= 2 MiB batches; the
one-launch handler step (k_handle_small) against on_message; the cgo entry
point gevws_decode_host_batch over two-segment host input.  Stream strategies: tests/test_properties.py."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import gev_amd
from gev_amd import _abi
from oracle import ws_oracle as wo
from tests._helpers import assert_matches_oracle, pack_streams
from tests.test_properties import frame, streams

pytestmark = pytest.mark.gpu

SETTINGS = settings(max_examples=300, deadline=None,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


@SETTINGS
@given(st.lists(streams, min_size=1, max_size=8), st.booleans())
def test_device_decode_equals_oracle(engine, ss, one_launch):
    arena, conns = pack_streams(ss)
    engine.set_tuning(_abi.TUNE_SMALL_BATCH, _abi.ONE_LAUNCH_MAX_BYTES if one_launch else 0)
    try:
        assert_matches_oracle(engine, arena, conns, f"one_launch={one_launch}")
    finally:
        engine.set_tuning(_abi.TUNE_SMALL_BATCH, _abi.ONE_LAUNCH_MAX_BYTES)


@pytest.fixture(scope="module")
def live_flag():
    import torch
    a = gev_amd.PinnedArena(4096)
    yield a
    torch.cuda.synchronize()
    a.close()


@settings(max_examples=150, deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture,
                                 HealthCheck.data_too_large])
@given(st.lists(streams, min_size=1, max_size=24), st.integers(1, 16))
def test_live_pass_decode_equals_oracle(engine, live_flag, ss, copies):
    """A live pass's form: with a completion flag set, the
    one-launch decode stages its input through up to 32 workgroups' tagged
    granules before the last one decodes -- on generated batches of up to
    384 connections, so both one-launch shapes (256 lanes / 64 KiB, 1 024
    lanes / 128 KiB) and, past them, the multi-kernel path run; bit-exact
    against the C oracle, and the flag carries this launch's number exactly
    when the decode was one launch."""
    batch = ss * copies
    arena, conns = pack_streams(batch)
    engine.set_completion_flag(live_flag, 64)
    try:
        assert_matches_oracle(engine, arena, conns, f"{len(batch)} connections, {len(arena)} bytes")
        one = len(batch) <= _abi.ONE_LAUNCH_MAX_CONNS and len(arena) <= _abi.ONE_LAUNCH_MAX_BYTES
        assert (engine.completion_seq > 0) == one
        if one:
            assert int(live_flag.host[64:68].view(np.uint32)[0]) == engine.completion_seq
    finally:
        engine.set_completion_flag(None)


@SETTINGS
@given(st.binary(min_size=1, max_size=600), st.binary(min_size=4, max_size=4), st.integers(0, 1 << 20),
       st.integers(0, 15))
def test_device_cipher_equals_bytewise(engine, payload, mask, offset, align):
    import torch
    buf = torch.zeros(align + len(payload) + 64, dtype=torch.uint8, device=torch.device("cuda", engine.device))
    buf[align:align + len(payload)] = torch.from_numpy(np.frombuffer(payload, np.uint8).copy()).to(buf.device)
    engine.cipher_(buf, mask, offset, nbytes=len(payload), byte_offset=align)
    torch.cuda.synchronize()
    want = bytearray(payload)
    wo.cipher_bytewise(want, mask, offset)
    got = buf.cpu().numpy().tobytes()
    assert got[align:align + len(payload)] == bytes(want)
    assert got[:align] == b"\0" * align and got[align + len(payload):] == b"\0" * 64


@st.composite
def out_frames(draw):
    """Records for the encode (OUT_FRAME_DTYPE) over one payload arena: any
    FIN / RSV / opcode / MASK bit and key, lengths across the 7-, 16- and
    64-bit forms, payloads at any alignment (overlapping ones too)."""
    n = draw(st.integers(0, 24))
    lens = [draw(st.one_of(st.integers(0, 300), st.sampled_from([125, 126, 65535, 65536]), st.integers(0, 70000)))
            for _ in range(n)]
    arena_len = sum(lens) + 64
    fr = np.zeros(n, gev_amd.OUT_FRAME_DTYPE)
    for i, L in enumerate(lens):
        fr[i]["fin"] = draw(st.integers(0, 1))
        fr[i]["rsv"] = draw(st.integers(0, 7))
        fr[i]["opcode"] = draw(st.integers(0, 15))
        fr[i]["masked"] = draw(st.integers(0, 1))
        fr[i]["mask"] = np.frombuffer(draw(st.binary(min_size=4, max_size=4)), np.uint8)
        fr[i]["length"] = L
        fr[i]["payload_len"] = L
        fr[i]["payload_off"] = draw(st.integers(0, arena_len - L))
    seed = draw(st.integers(0, 2**32 - 1))
    payload = np.random.default_rng(seed).integers(0, 256, arena_len, dtype=np.uint8)
    return fr, payload


@settings(max_examples=150, deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture,
                                 HealthCheck.data_too_large])
@given(out_frames())
def test_device_encode_equals_oracle(engine, case):
    """FrameToBytes (frame.go:274-278 over write.go:48-84) on the device equals
    oracle/ws_ref.c's encode: wire bytes and every frame's wire offset."""
    import torch
    from oracle import ref
    fr, payload = case
    d_pay = torch.from_numpy(np.concatenate([payload, np.zeros(16, np.uint8)])).to(torch.device("cuda", engine.device))
    wire, off = engine.encode(fr, d_pay)
    want, woff = ref.encode_batch(fr, payload)
    assert np.array_equal(wire.cpu().numpy(), want)
    assert np.array_equal(off, woff)


@st.composite
def client_frame(draw):
    """A client frame the handler step answers or ignores: text (any bytes,
    valid UTF-8 or not), binary, continuation, ping / pong, close with no
    body, one byte, or any 16-bit code plus any reason, reserved opcodes."""
    kind = draw(st.sampled_from(["data", "ping", "close", "other"]))
    key = draw(st.binary(min_size=4, max_size=4))
    masked = draw(st.booleans())
    if kind == "data":
        op = draw(st.sampled_from([wo.OP_TEXT, wo.OP_BINARY, 0]))
        body = draw(st.one_of(st.binary(max_size=300), st.text(max_size=80).map(lambda t: t.encode())))
        return wo.encode_frame(body, op, draw(st.booleans()), 0, masked, key)
    if kind == "ping":
        return wo.encode_frame(draw(st.binary(max_size=125)), draw(st.sampled_from([0x9, 0xA])), True, 0, masked, key)
    if kind == "close":
        body = draw(st.one_of(st.just(b""), st.binary(min_size=1, max_size=1),
                              st.builds(lambda c, r: c.to_bytes(2, "big") + r, st.integers(0, 65535),
                                        st.one_of(st.binary(max_size=60), st.text(max_size=30).map(lambda t: t.encode())))))
        return wo.encode_frame(body[:125], wo.OP_CLOSE, True, 0, masked, key)
    return wo.encode_frame(draw(st.binary(max_size=20)), draw(st.sampled_from([0x3, 0x7, 0xB, 0xF])), True, 0,
                           masked, key)


@settings(max_examples=150, deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(st.lists(st.lists(client_frame(), min_size=1, max_size=12), min_size=1, max_size=6),
       st.sampled_from([_abi.HANDLER_NONE, _abi.HANDLER_ECHO_BINARY, _abi.HANDLER_ECHO_TEXT]))
def test_device_dispatch_equals_oracle(engine, conns_frames, policy):
    """HandlerWrap.OnMessage + util.HandleClose / HandlePing / HandlePong
    (wrap.go:38-90, util.go:27-85) on the device, then FrameToBytes of the
    replies: wire bytes, reply map and the shutdown count equal
    oracle/ws_oracle.on_message's over the decoded frames."""
    import torch
    streams = [b"".join(fs) for fs in conns_frames]
    arena, conns = pack_streams(streams)
    dev = torch.device("cuda", engine.device)
    d_in = torch.zeros(len(arena) + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    d_in[: len(arena)] = torch.from_numpy(np.frombuffer(arena, np.uint8).copy()).to(dev)
    nf = sum(len(fs) for fs in conns_frames)
    out = engine.decode(d_in, len(arena), torch.from_numpy(conns.copy()).to(dev), conns.shape[0], aux_slots=nf + 1)
    wire, reply_of, ds = engine.serve(out, policy)
    want, shut, reps, k = b"", 0, [], 0
    for s in streams:
        for fr in wo.decode_stream(s).frames:
            r, sd = wo.on_message(fr.header, fr.payload, policy)
            shut += sd
            reps.append(-1 if r is None else k)
            if r is not None:
                want += r
                k += 1
    assert int(ds["errors"]) == shut and int(ds["frames"]) == k
    assert list(reply_of) == reps
    assert wire.cpu().numpy().tobytes() == want


@settings(max_examples=100, deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture,
                                 HealthCheck.data_too_large])
@given(st.lists(st.tuples(st.lists(frame(), min_size=1, max_size=8), st.integers(0, 13)), min_size=1, max_size=4),
       st.sampled_from([0, 1 << 30]), st.data())
def test_protocol_over_rings_equals_oracle(engine, conns_frames, zero_copy_max, data):
    """The host mirror of websocket.Protocol (protocol.go:38-62, driven as
    connection.go:208-251 drives it) over ring buffers fed in arbitrary
    chunks, with batched passes between reads: every connection gets exactly
    the oracle's frames in order, and the bytes of its trailing incomplete
    frame stay in its ring (the completeness gate and the carry)."""
    proto = gev_amd.Protocol(engine)
    proto.set_zero_copy_max(zero_copy_max)
    try:
        n = len(conns_frames)
        conns = [gev_amd.Connection(upgraded=True) for _ in range(n)]
        rings = [gev_amd.RingBuffer(data.draw(st.sampled_from([16, 4096]))) for _ in range(n)]
        wires = [b"".join(fs) + b"".join(fs)[:cut] for fs, cut in conns_frames]  # + a cut-off frame prefix
        want = [wo.decode_stream(w).frames for w in wires]
        got = [[] for _ in range(n)]
        pos = [0] * n
        while any(pos[i] < len(wires[i]) for i in range(n)):
            for i in range(n):
                k = data.draw(st.integers(1, 400))
                chunk = wires[i][pos[i]:pos[i] + k]
                pos[i] += len(chunk)
                if chunk:
                    rings[i].write(chunk)
            if data.draw(st.booleans()):
                proto.unpacket_batch(conns, rings)
            for i in range(n):
                while True:
                    h, d = proto.unpacket(conns[i], rings[i])
                    if h is None:
                        break
                    got[i].append((bytes(h), d))
        for i in range(n):
            assert [g for g in got[i]] == [(f.header.pack(), f.payload) for f in want[i]], i
            assert rings[i].length() == len(wires[i]) - sum(f.header_len + f.header.length for f in want[i]), i
    finally:
        proto.close()


@st.composite
def long_stream(draw):
    """A connection long enough to split (>= 2 KiB): runs of small frames
    (masked or not, any length form), tiny 2-5 byte frames, an unmasked
    frame carrying a plausible inner frame chain (guesses inside it confirm
    on bytes that are not frame starts), noise, and an incomplete tail."""
    parts = []
    while sum(len(p) for p in parts) < 2048:
        kind = draw(st.sampled_from(["small", "tiny", "embedded", "noise"]))
        if kind == "small":
            parts.append(b"".join(draw(st.lists(frame(), min_size=1, max_size=40))))
        elif kind == "tiny":
            parts.append(b"".join(wo.encode_frame(b"\x00" * draw(st.integers(0, 3)), 2, True, 0, False)
                                  for _ in range(draw(st.integers(1, 60)))))
        elif kind == "embedded":
            inner = b"".join(draw(st.lists(frame(), min_size=1, max_size=30)))
            parts.append(wo.encode_frame(inner, 2, True, 0, False))
        else:
            parts.append(draw(st.binary(min_size=1, max_size=600)))
    return b"".join(parts) + draw(st.binary(max_size=10))


@settings(max_examples=80, deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture,
                                 HealthCheck.data_too_large, HealthCheck.large_base_example])
@given(st.lists(long_stream(), min_size=1, max_size=4), st.sampled_from([2, 4, 8, 16, 32]))
def test_split_walk_equals_oracle(engine, ss, lanes):
    """The split header walk (k_walk_split: lanes guess frame starts inside a
    stream, walk between guesses, and a connection whose segments do not meet
    exactly is re-walked serially) equals the serial chain -- the oracle --
    bit-exactly on generated long streams, for every lane count, with 1 KiB
    segments so that small streams split."""
    arena, conns = pack_streams(ss)
    engine.set_tuning(_abi.TUNE_SMALL_BATCH, 0)
    engine.set_tuning(_abi.TUNE_SPLIT_LANES, lanes)
    engine.set_tuning(_abi.TUNE_SPLIT_MIN_BYTES, 1024)
    try:
        assert_matches_oracle(engine, arena, conns, f"lanes={lanes}")
        assert engine.last_split_lanes == lanes
    finally:
        engine.set_tuning(_abi.TUNE_SPLIT_LANES, 0)
        engine.set_tuning(_abi.TUNE_SPLIT_MIN_BYTES, 16384)
        engine.set_tuning(_abi.TUNE_SMALL_BATCH, _abi.ONE_LAUNCH_MAX_BYTES)


def _masked_frames_np(rng, lens, masked, forms):
    """Frames with random payloads, XOR-masked with numpy (fast for MiBs)."""
    out = []
    for L, m, f in zip(lens, masked, forms):
        key = bytes(rng.integers(0, 256, 4, dtype=np.uint8))
        p = rng.integers(0, 256, L, dtype=np.uint8)
        if m:
            p = p ^ np.resize(np.frombuffer(key, np.uint8), L)
        out.append(wo.write_header(True, 0, 2, L, m, key, f) + p.tobytes())
    return out


@settings(max_examples=40, deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(st.integers(0, 2**32 - 1), st.booleans(), st.integers(64, 48 * 1024), st.integers(1, 40),
       st.sampled_from([0, 1, 2]), st.sampled_from([0, 8, 12]))
def test_unmask_paths_equal_oracle(engine, seed, equal, L, n_conns, variant, grid):
    """The payload unmask over batches of >= 2 MiB: equal-size frames of any
    length (the v3 windows and, with a capped grid, the per-XCD counter runs
    over frames that cross tiles at every alignment) or mixed sizes (v5's
    chunk -> frame map), masked and unmasked, any length form, every unmask
    variant and grid: bit-exact against the C oracle."""
    rng = np.random.default_rng(seed)
    n = max(2, (2 << 20) // (L + 14) + 1)
    lens = [L] * n if equal else [int(x) for x in rng.integers(0, 2 * L + 1, n)]
    masked = [True] * n if equal else [bool(x) for x in rng.integers(0, 2, n)]
    frames = _masked_frames_np(rng, lens, masked, [None] * n)
    per = -(-n // n_conns)
    streams = [b"".join(frames[i:i + per]) for i in range(0, n, per)]
    arena, conns = pack_streams(streams)
    engine.set_tuning(_abi.TUNE_UNMASK_VARIANT, variant)
    engine.set_tuning(_abi.TUNE_UNMASK_GRID, grid)
    try:
        assert_matches_oracle(engine, arena, conns, f"equal={equal} L={L} variant={variant} grid={grid}")
    finally:
        engine.set_tuning(_abi.TUNE_UNMASK_VARIANT, 0)
        engine.set_tuning(_abi.TUNE_UNMASK_GRID, 0)


@settings(max_examples=120, deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(st.lists(st.lists(client_frame(), min_size=1, max_size=12), min_size=1, max_size=6),
       st.sampled_from([_abi.HANDLER_NONE, _abi.HANDLER_ECHO_BINARY, _abi.HANDLER_ECHO_TEXT]),
       st.integers(0, 40))
def test_one_launch_handler_equals_oracle(engine, conns_frames, policy, slack):
    """gevws_handle_decoded_async's one-workgroup form (k_handle_small: a
    live pass's dispatch and FrameToBytes of the replies in ONE launch, its
    frame count read from the decode's summary on the device, with a frame
    bound above the decoded count) equals on_message's replies byte for
    byte, with the same reply map and summaries."""
    import torch
    streams = [b"".join(fs) for fs in conns_frames]
    arena, conns = pack_streams(streams)
    dev = torch.device("cuda", engine.device)
    d_in = torch.zeros(len(arena) + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    d_in[: len(arena)] = torch.from_numpy(np.frombuffer(arena, np.uint8).copy()).to(dev)
    want, shut, reps, k = b"", 0, [], 0
    for s in streams:
        for fr in wo.decode_stream(s).frames:
            r, sd = wo.on_message(fr.header, fr.payload, policy)
            shut += sd
            reps.append(-1 if r is None else k)
            if r is not None:
                want += r
                k += 1
    nf = len(reps)
    aux = max(nf, 1)
    out = engine.decode(d_in, len(arena), torch.from_numpy(conns.copy()).to(dev), conns.shape[0], aux_slots=aux)
    wire, reply_of, ds, es = engine.handle_decoded(out, policy, nf + slack, aux, len(want) + 64)
    assert int(ds["status"]) == 0 and int(es["status"]) == 0
    assert int(ds["frames"]) == k and int(ds["errors"]) == shut
    assert int(es["frames"]) == k and int(es["payload_bytes"]) == len(want)
    assert list(reply_of) == reps
    assert wire.cpu().numpy().tobytes() == want


@settings(max_examples=120, deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(st.lists(streams, min_size=1, max_size=8), st.sampled_from([0, 1 << 30]), st.data())
def test_decode_host_batch_equals_oracle(engine, ss, zero_copy_max, data):
    """gevws_decode_host_batch (the cgo entry point: each connection's bytes
    as the two PeekAll segments of a ring, split anywhere, connection.go:
    237-244; copies in and out, or zero-copy on mapped memory): per-connection
    frames / consumed / status, records, src_off relative to the stream and
    payloads equal the oracle's."""
    proto = gev_amd.Protocol(engine)
    proto.set_zero_copy_max(zero_copy_max)
    try:
        segs = []
        for s in ss:
            cut = data.draw(st.integers(0, len(s)))
            segs.append((s[:cut], s[cut:]))
        frames, payload, cout, summ = proto.decode_host(segs)
        total = 0
        for ci, s in enumerate(ss):
            want = wo.decode_stream(s)
            total += len(want.frames)
            assert int(cout["nframes"][ci]) == len(want.frames)
            assert int(cout["consumed"][ci]) == want.consumed
            assert int(cout["status"][ci]) == want.status
            for j, fr in enumerate(want.frames):
                f = frames[int(cout["first_frame"][ci]) + j]
                assert f.tobytes()[:16] == fr.header.pack()
                assert int(f["src_off"]) == fr.stream_pos + fr.header_len
                o = int(f["payload_off"])
                assert payload[o:o + fr.header.length].tobytes() == fr.payload
        assert summ.frames == total
    finally:
        proto.close()
