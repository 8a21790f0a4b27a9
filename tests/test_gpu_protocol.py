"""The C++ host mirror of websocket.Protocol (plugins/websocket/protocol.go:27-69)
driven like gev drives it, with every decode on the device.

Modelled on the reference's only hot-path test, example/websocket/
wsserver_test.go:101-133 (clients send masked text frames of 1-3072 random
bytes and expect them back), but without sockets: bytes arrive in the
connection's ring buffer in read(2)-sized chunks (<= 64 KiB, eventloop.go:15),
and Connection.handlerProtocol (connection.go:208-218) calls UnPacket until it
returns (nil, nil).  Expected frames come from the oracle."""
import numpy as np
import pytest

import gev_amd
from oracle import ws_oracle as wo

pytestmark = pytest.mark.gpu


def _client_frames(rng, n):
    out = []
    for _ in range(n):
        sz = int(rng.integers(1, 3 * 1024 + 1))  # wsserver_test.go:112
        data = bytes(rng.integers(0, 256, sz, dtype=np.uint8))
        out.append((data, wo.encode_frame(data, wo.OP_TEXT, True, 0, True,
                                          bytes(rng.integers(0, 256, 4, dtype=np.uint8)))))
    return out


def test_echo_over_ring_buffers(engine):
    rng = np.random.default_rng(21)
    proto = gev_amd.Protocol(engine)
    n_conns = 100
    conns = [gev_amd.Connection(upgraded=True) for _ in range(n_conns)]
    rings = [gev_amd.RingBuffer(4096) for _ in range(n_conns)]  # DefaultBufferSize (eventloop.go:16)
    sent = [_client_frames(rng, int(rng.integers(1, 20))) for _ in range(n_conns)]
    wires = [b"".join(w for _, w in s) for s in sent]
    got = [[] for _ in range(n_conns)]
    pos = [0] * n_conns

    def on_message(c, hdr, data):
        got[idx].append((hdr.opcode, hdr.fin, data))
        return data  # echo, like the test server's OnMessage

    while any(pos[i] < len(wires[i]) for i in range(n_conns)):
        for idx in range(n_conns):
            if pos[idx] >= len(wires[idx]):
                continue
            n = int(rng.integers(1, 65537))
            chunk = wires[idx][pos[idx]:pos[idx] + n]
            pos[idx] += len(chunk)
            rings[idx].write(chunk)
            replies = gev_amd.handler_protocol(proto, conns[idx], rings[idx], on_message)
            assert all(isinstance(r, bytes) for r in replies)
    for i in range(n_conns):
        assert [d for _, _, d in got[i]] == [d for d, _ in sent[i]], i
        assert all(op == wo.OP_TEXT and fin for op, fin, _ in got[i])
        assert rings[i].length() == 0


@pytest.mark.parametrize("zero_copy_max", [0, 1 << 30])
def test_batched_driver_matches_oracle(engine, zero_copy_max):
    """zero_copy_max 0: the pass copies in and out; 1 GiB: the kernels run on
    the mapped pinned staging and write into mapped host memory."""
    rng = np.random.default_rng(22)
    proto = gev_amd.Protocol(engine)
    proto.set_zero_copy_max(zero_copy_max)
    streams = []
    for _ in range(64):
        s = b""
        for _ in range(int(rng.integers(0, 15))):
            L = int(rng.integers(0, 4000))
            s += wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), int(rng.choice([0, 1, 2, 9, 10])),
                                 bool(rng.random() < .8), 0, bool(rng.random() < .9),
                                 bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
        s += bytes(rng.integers(0, 256, int(rng.integers(0, 10)), dtype=np.uint8))
        streams.append(s)
    conns = [gev_amd.Connection() for _ in streams]
    rings = []
    for s in streams:
        r = gev_amd.RingBuffer(64)
        r.write(b"\x00" * 40)   # force wrap-around: write, consume, write
        r.retrieve(40)
        r.write(s)
        rings.append(r)
    n = proto.unpacket_batch(conns, rings)
    assert n == sum(len(wo.decode_stream(s).frames) for s in streams)
    for c, r, s in zip(conns, rings, streams):
        want = wo.decode_stream(s)
        assert c.pending() == len(want.frames)
        for fr in want.frames:
            h, data = proto.unpacket(c, r)
            assert h is not None
            assert (bool(h.fin), h.rsv, h.opcode, bool(h.masked), bytes(h.mask), h.length) == (
                fr.header.fin, fr.header.rsv, fr.header.opcode, fr.header.masked, fr.header.mask, fr.header.length)
            assert data == fr.payload
        assert proto.unpacket(c, r) == (None, None)
        assert proto.last_status == gev_amd.NEED_MORE
        assert r.length() == len(s) - want.consumed
    st = proto.stats()
    assert st["zero_copy_passes"] == (st["device_passes"] if zero_copy_max else 0), st


@pytest.mark.parametrize("zero_copy_max", [0, 1 << 30])
def test_batch_begin_end_with_ring_writes_in_flight(engine, zero_copy_max):
    """gevws_protocol_unpacket_batch_begin / _end: the pass decodes the bytes
    buffered at _begin while the rings take more (an event loop reading its
    sockets during the pass); a second _begin in flight is refused; the
    frames come out exactly as the oracle decodes each part, and UnPacket
    ends a pass in flight before it answers."""
    rng = np.random.default_rng(23)
    proto = gev_amd.Protocol(engine)
    proto.set_zero_copy_max(zero_copy_max)

    def part():
        s = b""
        for _ in range(int(rng.integers(1, 8))):
            L = int(rng.integers(0, 3000))
            s += wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), 2, True, 0, True,
                                 bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
        return s
    first = [part() for _ in range(40)]
    second = [part() for _ in range(40)]
    conns = [gev_amd.Connection() for _ in first]
    rings = [gev_amd.RingBuffer(64) for _ in first]
    for r, s in zip(rings, first):
        r.write(s)
    assert proto.unpacket_batch_begin(conns, rings) == len(conns)
    for r, s in zip(rings, second):  # bytes arriving while the pass runs
        r.write(s)
    with pytest.raises(RuntimeError):
        proto.unpacket_batch_begin(conns, rings)
    n = proto.unpacket_batch_end()
    assert n == sum(len(wo.decode_stream(s).frames) for s in first)
    assert proto.unpacket_batch_end() == 0
    for c, r, s1, s2 in zip(conns, rings, first, second):
        want = wo.decode_stream(s1).frames + wo.decode_stream(s2).frames
        for fr in want:  # the first part from the pass, the second from UnPacket's own passes
            h, data = proto.unpacket(c, r)
            assert h is not None and h.length == fr.header.length and data == fr.payload
        assert proto.unpacket(c, r) == (None, None)
        assert r.length() == 0
    # UnPacket with a pass in flight: it ends the pass first
    for r, s in zip(rings, first):
        r.write(s)
    assert proto.unpacket_batch_begin(conns, rings) == len(conns)
    h, data = proto.unpacket(conns[0], rings[0])
    assert data == wo.decode_stream(first[0]).frames[0].payload
    assert conns[1].pending() == len(wo.decode_stream(first[1]).frames)


@pytest.mark.parametrize("zero_copy_max", [0, 1 << 30])
def test_pass_in_flight_then_decode_host_and_batch(engine, zero_copy_max):
    """gevws_decode_host_batch and gevws_protocol_unpacket_batch
    share the staging buffers with a pass begun by _begin; both finish that
    pass (its frames queued on its connections) before they stage their own,
    so begin -> decode_host -> end and begin -> unpacket_batch deliver every
    frame to the right connection."""
    rng = np.random.default_rng(29)
    proto = gev_amd.Protocol(engine)
    proto.set_zero_copy_max(zero_copy_max)

    def stream(k):
        return b"".join(wo.encode_frame(bytes(rng.integers(0, 256, int(rng.integers(0, 2000)), dtype=np.uint8)),
                                        2, True, 0, True, bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
                        for _ in range(k))
    first = [stream(int(rng.integers(1, 6))) for _ in range(24)]
    conns = [gev_amd.Connection() for _ in first]
    rings = [gev_amd.RingBuffer(64) for _ in first]
    for r, s in zip(rings, first):
        r.write(s)
    assert proto.unpacket_batch_begin(conns, rings) == len(conns)
    # a host decode in between: its own output is the oracle's ...
    other = [stream(3) + b"\x82\xfe", stream(1)]
    frames, payload, cout, summ = proto.decode_host([(s, b"") for s in other])
    want = [wo.decode_stream(s) for s in other]
    assert int(summ.frames) == sum(len(w.frames) for w in want)
    for j, w in enumerate(want):
        assert int(cout[j]["nframes"]) == len(w.frames)
        for k, fr in enumerate(w.frames):
            rec = frames[int(cout[j]["first_frame"]) + k]
            off = int(rec["payload_off"])
            assert bytes(payload[off:off + fr.header.length]) == fr.payload
    # ... and the pass in flight was delivered to its own connections
    assert proto.unpacket_batch_end() == 0
    for c, s in zip(conns, first):
        assert c.pending() == len(wo.decode_stream(s).frames)
    for c, r, s in zip(conns, rings, first):
        for fr in wo.decode_stream(s).frames:
            h, data = proto.unpacket(c, r)
            assert h is not None and data == fr.payload
        assert proto.unpacket(c, r) == (None, None)
    # begin -> unpacket_batch: the batch call ends the pass first instead of failing
    second = [stream(2) for _ in first]
    for r, s in zip(rings, second):
        r.write(s)
    assert proto.unpacket_batch_begin(conns[:12], rings[:12]) == 12
    proto.unpacket_batch(conns, rings)  # the first 12 hold frames now: the other 12 are decoded
    for c, r, s in zip(conns, rings, second):
        got = [proto.unpacket(c, r)[1] for _ in wo.decode_stream(s).frames]
        assert got == [fr.payload for fr in wo.decode_stream(s).frames]
        assert proto.unpacket(c, r) == (None, None)


def test_zero_copy_capacity_retry(engine):
    """A zero-copy pass sizes its host outputs from an estimate (~1 frame per
    48 input bytes); a run of empty frames (6 bytes each) exceeds it, the pass
    reports GEVWS_ERR_CAPACITY and is re-run once with the exact sizes."""
    proto = gev_amd.Protocol(engine)
    c, r = gev_amd.Connection(), gev_amd.RingBuffer(1 << 16)
    w = b"".join(wo.encode_frame(b"", 2, True, 0, True, bytes([i & 255, 1, 2, 3])) for i in range(3000))
    tail = bytes([0x82, 0x7F, 0, 0, 0])  # 5 bytes of a 64-bit-length header: (nil, nil), read.go:20-23
    w += wo.encode_frame(b"end", 1, True, 0, True, b"\x09\x08\x07\x06") + tail
    r.write(w)
    got = gev_amd.handler_protocol(proto, c, r, lambda cc, h, d: (h.opcode, d))
    assert got == [(2, b"")] * 3000 + [(1, b"end")]
    st = proto.stats()
    assert st["device_passes"] == 1 and st["zero_copy_passes"] == 1, st
    assert r.length() == len(tail)


def test_not_upgraded_and_poison(engine):
    proto = gev_amd.Protocol(engine)
    c = gev_amd.Connection(upgraded=False)
    r = gev_amd.RingBuffer()
    r.write(wo.encode_frame(b"hi", 1, True, 0, True, b"\x01\x02\x03\x04"))
    assert proto.unpacket(c, r) == (None, None)
    assert proto.last_status == gev_amd.ERR_NOT_UPGRADED
    c.set_upgraded(True)
    r.write(bytes([0x82, 0xFF, 0x80, 0, 0, 0, 0, 0, 0, 5, 1, 2, 3, 4]) + b"hello")
    h, d = proto.unpacket(c, r)
    assert d == b"hi"
    for _ in range(2):   # sticky: logged and (nil, nil) on every later call
        assert proto.unpacket(c, r) == (None, None)
        assert proto.last_status == gev_amd.ERR_LEN_MSB


def test_need_more_then_complete(engine):
    proto = gev_amd.Protocol(engine)
    c = gev_amd.Connection()
    r = gev_amd.RingBuffer(16)
    w = wo.encode_frame(bytes(range(200)), 2, True, 0, True, b"\x09\x08\x07\x06")
    for cut in (1, 5, 6, 7, 8, 100, len(w) - 1):
        r.write(w[:cut])
        assert proto.unpacket(c, r) == (None, None)
        assert proto.last_status == gev_amd.NEED_MORE
        assert r.length() == cut
        r.retrieve(cut)
    r.write(w)
    h, d = proto.unpacket(c, r)
    assert d == bytes(range(200)) and h.length == 200 and r.length() == 0


@pytest.mark.parametrize("zero_copy_max", [0, 1 << 30])
def test_decode_host_batch_two_segments(engine, zero_copy_max):
    """gevws_decode_host_batch (the cgo entry point): each connection's bytes
    arrive as the two PeekAll segments of a wrapped ring (connection.go:237-244).
    Both pass forms: copies in and out, and zero-copy on mapped pinned memory
    with a CPU copy into the caller's buffers."""
    from tests._helpers import random_stream
    rng = np.random.default_rng(23)
    proto = gev_amd.Protocol(engine)
    proto.set_zero_copy_max(zero_copy_max)
    streams = [random_stream(rng, int(rng.integers(0, 20))) for _ in range(50)]
    segs = []
    for s in streams:
        cut = int(rng.integers(0, len(s) + 1))
        segs.append((s[:cut], s[cut:]))
    frames, payload, cout, summ = proto.decode_host(segs)
    for ci, s in enumerate(streams):
        want = wo.decode_stream(s)
        assert int(cout["nframes"][ci]) == len(want.frames)
        assert int(cout["consumed"][ci]) == want.consumed
        assert int(cout["status"][ci]) == want.status
        for j, fr in enumerate(want.frames):
            f = frames[int(cout["first_frame"][ci]) + j]
            assert f.tobytes()[:16] == fr.header.pack()
            assert int(f["src_off"]) == fr.stream_pos + fr.header_len
            o = int(f["payload_off"])
            assert payload[o:o + fr.header.length].tobytes() == fr.payload
    assert summ.frames == sum(len(wo.decode_stream(s).frames) for s in streams)
    assert proto.stats()["zero_copy_passes"] == (1 if zero_copy_max else 0)


def test_decode_host_stream_single_connection(engine):
    import ctypes
    from gev_amd import _abi
    rng = np.random.default_rng(24)
    from tests._helpers import random_stream
    proto = gev_amd.Protocol(engine)
    s = random_stream(rng, 30)
    cut = len(s) // 3
    a = np.frombuffer(s[:cut], np.uint8).copy()
    b = np.frombuffer(s[cut:], np.uint8).copy()
    frames = np.zeros(len(s), gev_amd.FRAME_DTYPE)
    payload = np.zeros(len(s) * 20 + 64, np.uint8)
    cout = np.zeros(1, gev_amd.CONN_OUT_DTYPE)
    summ = _abi.Summary()
    n = gev_amd.lib.gevws_decode_host_stream(proto._p, a.ctypes.data, a.size, b.ctypes.data, b.size,
                                             frames.ctypes.data, frames.size, payload.ctypes.data, payload.size,
                                             cout.ctypes.data, ctypes.byref(summ))
    want = wo.decode_stream(s)
    assert n == len(want.frames) and int(cout["consumed"][0]) == want.consumed
    for f, fr in zip(frames[:n], want.frames):
        o = int(f["payload_off"])
        assert f.tobytes()[:16] == fr.header.pack() and payload[o:o + fr.header.length].tobytes() == fr.payload


XNET_REQUEST = (b"GET / HTTP/1.1\r\nHost: localhost:1834\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                b"Sec-WebSocket-Key: x3JJHMbDL1EzLkh9GBhXDw==\r\nOrigin: ws://localhost:1834\r\n"
                b"Sec-WebSocket-Version: 13\r\n\r\n")


def _wrap_on_message(got):
    """HandlerWrap.OnMessage (wrap.go:38-44): a (nil, out) from UnPacket is the
    handshake response and is sent back as-is; frames are echoed."""
    def on_message(c, hdr, data):
        if hdr is None:
            return data
        got.append(data)
        return data
    return on_message


def test_handshake_then_frames_in_chunks(engine):
    """protocol.go:27-37 end to end: the upgrade request and the first frames
    arrive together, in small read(2) chunks; the 101 response is the first
    reply, then every frame is decoded on the device and echoed."""
    from oracle import ws_handshake as wh
    rng = np.random.default_rng(33)
    proto = gev_amd.Protocol(engine, gev_amd.Upgrader())
    c = gev_amd.Connection(upgraded=False)
    r = gev_amd.RingBuffer(64)
    sent = _client_frames(rng, 12)
    wire = XNET_REQUEST + b"".join(w for _, w in sent)
    got, replies, pos = [], [], 0
    on_message = _wrap_on_message(got)
    while pos < len(wire):
        n = int(rng.integers(1, 700))
        r.write(wire[pos:pos + n])
        pos += n
        replies += gev_amd.handler_protocol(proto, c, r, on_message)
    want_101 = wh.upgrade(XNET_REQUEST, b"").out
    assert replies[0] == want_101 and c.upgraded
    assert c.handshake().http_code == 101
    assert got == [d for d, _ in sent] and replies[1:] == got
    assert r.length() == 0


def test_handshake_rejected_then_retried(engine):
    """A bad request is answered with the error response and the connection
    stays un-upgraded (protocol.go:31-34 returns (nil, out)); a later good
    request upgrades it."""
    from oracle import ws_handshake as wh
    proto = gev_amd.Protocol(engine, gev_amd.Upgrader())
    c = gev_amd.Connection(upgraded=False)
    r = gev_amd.RingBuffer(256)
    bad = XNET_REQUEST.replace(b"Sec-WebSocket-Version: 13", b"Sec-WebSocket-Version: 8")
    replies = gev_amd.handler_protocol(proto, c, r, _wrap_on_message([]))
    assert replies == [] and proto.last_status == gev_amd.ERR_HANDSHAKE   # empty ring: malformed, silent
    r.write(bad)
    replies = gev_amd.handler_protocol(proto, c, r, _wrap_on_message([]))
    assert replies == [wh.upgrade(bad, b"").out] and not c.upgraded and r.length() == 0
    assert replies[0].startswith(b"HTTP/1.1 426 Upgrade Required\r\n")
    # the loop's last UnPacket ran the upgrade on the now empty ring: (nil, nil)
    assert c.handshake().error == gev_amd._abi.HS_MALFORMED_REQUEST
    frame = wo.encode_frame(b"hello", wo.OP_TEXT, True, 0, True, b"\x01\x02\x03\x04")
    r.write(XNET_REQUEST + frame)
    got = []
    replies = gev_amd.handler_protocol(proto, c, r, _wrap_on_message(got))
    assert c.upgraded and got == [b"hello"] and replies[1:] == [b"hello"]


def test_large_frame_in_read_sized_chunks_costs_one_pass(engine):
    """A 1 MiB frame arriving in 64 KiB reads (connection.go:220-251,
    eventloop.go:15): every UnPacket before the last read is answered by the
    carried completeness gate (protocol.go:47, 59-61) without a device pass;
    the read that completes it costs exactly one pass."""
    rng = np.random.default_rng(31)
    proto = gev_amd.Protocol(engine)
    c, r = gev_amd.Connection(), gev_amd.RingBuffer(4096)
    data = bytes(rng.integers(0, 256, 1 << 20, dtype=np.uint8))
    w = wo.encode_frame(data, wo.OP_BINARY, True, 0, True, b"\x11\x22\x33\x44")
    w2 = wo.encode_frame(b"tail", wo.OP_TEXT, True, 0, True, b"\x01\x02\x03\x04")
    stream = w + w2
    chunks = [stream[i:i + 65536] for i in range(0, len(stream), 65536)]
    got = []
    for ch in chunks:
        r.write(ch)
        got += gev_amd.handler_protocol(proto, c, r, lambda cc, h, d: d)
    st = proto.stats()
    assert got == [data, b"tail"]
    assert st["device_passes"] == 1, st
    assert st["gated"] >= len(chunks) - 1, st
    assert r.length() == 0


def test_carry_survives_deliveries_and_external_consumption(engine):
    """The carried gate is tied to the ring's read position: frames delivered
    by UnPacket keep it exact, bytes consumed by anyone else invalidate it."""
    rng = np.random.default_rng(32)
    proto = gev_amd.Protocol(engine)
    c, r = gev_amd.Connection(), gev_amd.RingBuffer(64)
    frames = [bytes(rng.integers(0, 256, int(n), dtype=np.uint8)) for n in (10, 300, 5000, 0, 70000, 3)]
    wire = b"".join(wo.encode_frame(d, 2, True, 0, True, bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
                    for d in frames)
    got, pos = [], 0
    while pos < len(wire):
        n = int(rng.integers(1, 9000))
        r.write(wire[pos:pos + n])
        pos += n
        got += gev_amd.handler_protocol(proto, c, r, lambda cc, h, d: d if d else None)
    assert got == [d for d in frames if d]
    # external consumption: a partial frame is dropped by the caller, then a
    # short complete frame follows; the stale carry must not hide it
    big = wo.encode_frame(bytes(1000), 2, True, 0, True, b"\x01\x02\x03\x04")
    r.write(big[:500])
    assert proto.unpacket(c, r) == (None, None)
    r.retrieve(500)
    small = wo.encode_frame(b"abc", 1, True, 0, True, b"\x05\x06\x07\x08")
    r.write(small + bytes(6))
    h, d = proto.unpacket(c, r)
    assert d == b"abc" and h.opcode == 1


def test_duplicate_connection_in_one_batch(engine):
    """the same (connection, ring) twice in one UnPacketBatch is
    decoded once; frames are delivered once and stay aligned."""
    proto = gev_amd.Protocol(engine)
    c, r = gev_amd.Connection(), gev_amd.RingBuffer(256)
    w = [wo.encode_frame(bytes([i]) * (50 + i), 2, True, 0, True, bytes([i, 1, 2, 3])) for i in range(5)]
    r.write(b"".join(w) + bytes(3))
    n = proto.unpacket_batch([c, c, c], [r, r, r])
    assert n == 5 and c.pending() == 5
    for i in range(5):
        h, d = proto.unpacket(c, r)
        assert d == bytes([i]) * (50 + i)
    assert proto.unpacket(c, r) == (None, None) and r.length() == 3
    assert proto.stats()["device_passes"] == 1


def _control_mix(rng, n):
    """Client frames of the wsserver_test.go shape (masked text, 1-3072 random
    bytes) with masked control frames between them: pings and pongs (0-125
    bytes), and closes with valid, reserved, unknown and application codes,
    UTF-8 and non-UTF-8 reasons, and empty bodies (util.go:27-85)."""
    out = []
    codes = [1000, 1001, 1002, 1003, 1005, 1006, 1007, 1011, 1015, 1016, 2999, 3000, 4999, 999, 5000]
    for _ in range(n):
        r = rng.random()
        key = bytes(rng.integers(0, 256, 4, dtype=np.uint8))
        if r < 0.55:
            p = bytes(rng.integers(0, 256, int(rng.integers(1, 3073)), dtype=np.uint8))
            out.append(wo.encode_frame(p, wo.OP_TEXT, True, 0, True, key))
        elif r < 0.75:
            p = bytes(rng.integers(0, 256, int(rng.integers(0, 126)), dtype=np.uint8))
            out.append(wo.encode_frame(p, wo.OP_PING, True, 0, True, key))
        elif r < 0.85:
            p = bytes(rng.integers(0, 256, int(rng.integers(0, 126)), dtype=np.uint8))
            out.append(wo.encode_frame(p, wo.OP_PONG, True, 0, True, key))
        else:
            k = rng.random()
            if k < 0.15:
                body = b""
            else:
                reason = "bye ü".encode() if k < 0.6 else bytes([0xC3, 0x28, 0x41])
                body = int(rng.choice(codes)).to_bytes(2, "big") + reason[: int(rng.integers(0, 6))]
            out.append(wo.encode_frame(body, wo.OP_CLOSE, True, 0, True, key))
    return out


@pytest.mark.parametrize("policy", [wo.HANDLER_ECHO_TEXT, wo.HANDLER_ECHO_BINARY, wo.HANDLER_NONE])
@pytest.mark.parametrize("zero_copy_max", [0, 1 << 30])
def test_device_handler_replies_match_oracle(engine, policy, zero_copy_max):
    """gevws_protocol_set_handler: every pass runs HandlerWrap.OnMessage
    (wrap.go:38-90) on the device -- close -> HandleClose reply + ShutdownWrite,
    ping -> pong, pong -> ping, data -> the policy's echo -- and each frame's
    reply (gevws_protocol_reply) equals oracle/ws_oracle.on_message's, byte for
    byte, over many connections fed in read(2)-sized chunks."""
    rng = np.random.default_rng(31 + policy)
    proto = gev_amd.Protocol(engine)
    proto.set_zero_copy_max(zero_copy_max)
    proto.set_handler(policy)
    streams = [b"".join(_control_mix(rng, int(rng.integers(1, 30)))) for _ in range(64)]
    conns = [gev_amd.Connection() for _ in streams]
    rings = [gev_amd.RingBuffer(4096) for _ in streams]
    pos = [0] * len(streams)
    got = [[] for _ in streams]
    while any(p < len(s) for p, s in zip(pos, streams)):
        for i, s in enumerate(streams):
            k = int(rng.integers(1, 9000))
            rings[i].write(s[pos[i]:pos[i] + k])
            pos[i] = min(len(s), pos[i] + k)
        proto.unpacket_batch(conns, rings)
        for i in range(len(streams)):
            h, data = proto.unpacket(conns[i], rings[i])
            while h is not None:
                got[i].append((h.opcode, data, proto.reply(conns[i])))
                h, data = proto.unpacket(conns[i], rings[i])
    n = 0
    for s, g in zip(streams, got):
        want = wo.decode_stream(s).frames
        assert len(g) == len(want)
        for (op, data, (rep, shut)), fr in zip(g, want):
            assert op == fr.header.opcode and data == fr.payload
            wrep, wshut = wo.on_message(fr.header, fr.payload, policy)
            assert rep == wrep and shut == wshut, (fr.header, fr.payload[:16], rep, wrep)
            n += 1
    assert n > 500
    st = proto.stats()
    assert st["handler_passes"] > 0
    # zero-copy passes chain the handler behind the decode (one synchronisation)
    # and wait on the kernels' completion flag instead of the stream
    assert (st["chained_handler_passes"] > 0) == (zero_copy_max > 0)
    assert (st["signalled_passes"] > 0) == (zero_copy_max > 0)


def _handler_pass_matches_oracle(engine, proto, streams, policy):
    conns = [gev_amd.Connection() for _ in streams]
    rings = [gev_amd.RingBuffer(len(s) + 16) for s in streams]
    for r, s in zip(rings, streams):
        r.write(s)
    proto.unpacket_batch(conns, rings)
    n = 0
    for c, r, s in zip(conns, rings, streams):
        want = wo.decode_stream(s).frames
        for fr in want:
            h, data = proto.unpacket(c, r)
            assert h is not None and h.opcode == fr.header.opcode and data == fr.payload
            assert proto.reply(c) == wo.on_message(fr.header, fr.payload, policy)
            n += 1
        assert proto.unpacket(c, r)[0] is None
    return n


def test_chained_handler_falls_back_exactly(engine):
    """The chained handler step is sized from the staged bytes; when that
    guess is wrong the pass re-runs the step with the exact sizes: (1) a
    zero-copy decode that misses its frame estimate (1 000 empty frames: the
    decode itself re-runs, the chained step saw a failed decode), (2) more
    close frames in one pass than the 4 096 aux slots the chain reserves.
    Replies equal oracle/ws_oracle.on_message's either way."""
    policy = wo.HANDLER_ECHO_TEXT
    proto = gev_amd.Protocol(engine)
    proto.set_zero_copy_max(1 << 30)
    proto.set_handler(policy)
    key = b"\x0a\x0b\x0c\x0d"
    empties = b"".join(wo.encode_frame(b"", wo.OP_TEXT, True, 0, True, key) for _ in range(1000))
    n = _handler_pass_matches_oracle(engine, proto, [empties, empties[:600]], policy)
    assert n == 1100
    body = (1000).to_bytes(2, "big") + b"r" * 121
    closes = b"".join(wo.encode_frame(body, wo.OP_CLOSE, True, 0, True, key) for _ in range(4097))
    assert _handler_pass_matches_oracle(engine, proto, [closes], policy) == 4097
    st = proto.stats()
    assert st["chained_handler_passes"] == 2 and st["handler_passes"] == 2
    # the first pass and its re-run decode signal (one-launch kernels); the
    # 528 KB second pass takes the multi-kernel decode and synchronises
    assert st["signalled_passes"] == 2


def test_device_handler_off_by_default(engine):
    proto = gev_amd.Protocol(engine)
    c, r = gev_amd.Connection(), gev_amd.RingBuffer(4096)
    r.write(wo.encode_frame(b"ping", wo.OP_PING, True, 0, True, b"\x01\x02\x03\x04"))
    h, data = proto.unpacket(c, r)
    assert h is not None and data == b"ping"
    with pytest.raises(RuntimeError):
        proto.reply(c)
    with pytest.raises(ValueError):
        proto.set_handler(7)


def test_reply_follows_the_frames_own_pass(engine):
    """gevws_protocol_reply answers from the pass that decoded the frame
    (ADVICE r3): a ping queued while the handler was off has no answer even
    after set_handler() (not an OK with no pong), and a frame decoded while the
    handler was on keeps its pong after the handler is turned off."""
    key = b"\x01\x02\x03\x04"
    ping = wo.encode_frame(b"ping", wo.OP_PING, True, 0, True, key)
    proto = gev_amd.Protocol(engine)
    c, r = gev_amd.Connection(), gev_amd.RingBuffer(4096)
    r.write(ping + ping)
    proto.unpacket_batch([c], [r])  # both pings queued, no handler ran
    proto.set_handler(wo.HANDLER_ECHO_TEXT)
    h, data = proto.unpacket(c, r)
    assert h is not None and data == b"ping"
    with pytest.raises(RuntimeError):
        proto.reply(c)
    proto.unpacket(c, r)
    # decoded with the handler on, handed out after it is turned off
    r.write(ping)
    proto.unpacket_batch([c], [r])
    proto.set_handler(-1)
    h, data = proto.unpacket(c, r)
    assert h is not None and data == b"ping"
    fr = wo.decode_stream(ping).frames[0]
    assert proto.reply(c) == wo.on_message(fr.header, fr.payload, wo.HANDLER_ECHO_TEXT)


def test_pass_timeline_small_zero_copy_pass(engine):
    """gevws_protocol_get_timeline: a small zero-copy pass
    (one launch, answered by the completion flag) reports its host phases and
    the kernel's own GPU time from its tick stamps; the frames are still the
    oracle's."""
    rng = np.random.default_rng(5)
    proto = gev_amd.Protocol(engine)
    conns = [gev_amd.Connection() for _ in range(100)]
    rings, streams = [], []
    for c in conns:
        s = b"".join(wo.encode_frame(bytes(rng.integers(0, 256, 128, dtype=np.uint8)), 1, True, 0, True,
                                     bytes(rng.integers(0, 256, 4, dtype=np.uint8))) for _ in range(2))
        r = gev_amd.RingBuffer(4096)
        r.write(s)
        rings.append(r)
        streams.append(s)
    for k in range(3):
        assert proto.unpacket_batch(conns, rings) == 200
        for c, r, s in zip(conns, rings, streams):
            for fr in wo.decode_stream(s).frames:
                h, data = proto.unpacket(c, r)
                assert data == fr.payload
            r.write(s)
    t = proto.timeline()
    assert t["passes"] == 3 and t["signalled"] == 3, t
    for k in ("ns_select", "ns_stage", "ns_launch", "ns_wait", "ns_deliver", "ns_gpu_decode"):
        assert t[k] > 0, (k, t)
    assert t["ns_gpu_decode"] < t["ns_wait"] < 3 * 10**9, t  # the kernel ran inside the wait
    assert t["ns_gpu_handler"] == 0 and t["ns_gpu_gap"] == 0


def test_pass_timeline_with_device_handler(engine):
    """The timeline's handler slot: a small zero-copy pass with the
    device handler on chains the one-launch handler step behind the decode;
    both kernels stamp their ticks, so the pass reports the handler's GPU time
    and the gap between the two kernels (>= 0), and every pass is answered by
    the completion flag.  The replies are still oracle/ws_oracle.on_message's."""
    rng = np.random.default_rng(6)
    policy = wo.HANDLER_ECHO_TEXT
    proto = gev_amd.Protocol(engine)
    proto.set_handler(policy)
    conns = [gev_amd.Connection() for _ in range(16)]  # ~30 KB: <= 1 024 records, the one-launch handler
    rings, streams = [], []
    for c in conns:
        s = b"".join(_control_mix(rng, 3))
        r = gev_amd.RingBuffer(4096)
        r.write(s)
        rings.append(r)
        streams.append(s)
    for k in range(3):
        proto.unpacket_batch(conns, rings)
        for c, r, s in zip(conns, rings, streams):
            for fr in wo.decode_stream(s).frames:
                h, data = proto.unpacket(c, r)
                assert data == fr.payload
                assert proto.reply(c) == wo.on_message(fr.header, fr.payload, policy)
            r.write(s)
    t = proto.timeline()
    st = proto.stats()
    assert st["chained_handler_passes"] == 3 and st["handler_passes"] == 3, st
    assert t["passes"] == 3 and t["signalled"] == 3, t
    assert t["ns_gpu_decode"] > 0 and t["ns_gpu_handler"] > 0 and t["ns_gpu_gap"] >= 0, t
    assert t["ns_gpu_decode"] + t["ns_gpu_handler"] < t["ns_wait"] + t["ns_launch"], t


@pytest.mark.parametrize("mode", ["default", "all", "normal"])
def test_contexts_cycle_stream_priorities(mode, monkeypatch):
    """One context per event loop: successive contexts on a device cycle their
    stream's priority (each level has its own hardware queues, so eight loops'
    passes run side by side instead of three at a time,
    profiles/r05/r05u_queue_probe.jsonl).  By default only over the normal
    level and those below it -- a context never outranks the application's
    own normal-priority work; GEVWS_STREAM_PRIORITIES=all adds the
    levels above, =normal keeps every context at 0.  Each still decodes
    exactly."""
    import torch

    if mode != "default":
        monkeypatch.setenv("GEVWS_STREAM_PRIORITIES", mode)
    engines = [gev_amd.Engine(0) for _ in range(6)]
    prios = [torch.cuda.ExternalStream(int(gev_amd.lib.gevws_ctx_stream(e._ctx)), device="cuda:0").priority
             for e in engines]
    if mode == "normal":
        assert set(prios) == {0}, prios
    elif mode == "default":
        assert min(prios) == 0 and len(set(prios)) >= 2, prios  # (the box's range is -1 .. 1)
    else:
        assert min(prios) < 0 < max(prios) and len(set(prios)) >= 3, prios
    rng = np.random.default_rng(9)
    for e in engines:
        proto = gev_amd.Protocol(e)
        c, r = gev_amd.Connection(), gev_amd.RingBuffer(4096)
        frames = _client_frames(rng, 5)
        r.write(b"".join(w for _, w in frames))
        assert proto.unpacket_batch([c], [r]) == 5
        for data, _ in frames:
            assert proto.unpacket(c, r)[1] == data
        proto.close()  # before its engine (Protocol.close)
        e.close()
