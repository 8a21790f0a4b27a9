"""Property-based checks (CPU, hypothesis) of the decode contract the HIP path
is held to, with shrinking to a minimal failing
stream:

* the two oracle restatements -- oracle/ws_oracle.py (bytewise Python) and
  oracle/ws_ref.c (the Go word-loop Cipher) -- decode every generated stream
  identically: frames, payloads, consumed bytes, status (read.go:19-84,
  protocol.go:38-62, connection.go:208-218);
* the completeness gate (protocol.go:47 + the ringbuffer contract, §8a a7): a
  prefix of a stream decodes to a prefix of its frames, and the leading frames
  whose h + L bytes lie inside the prefix, each starting >= 6 bytes before its
  end (read.go:20-23), are emitted;
* the product library's host exports (the boundary's per-frame calls, §8b
  items 1-2): gevws_parse_header_ring over a ring wrapped at any point equals
  the oracle's read_header of the joined bytes, and gevws_cipher equals the
  bytewise ws.Cipher at any offset;
* the host ring the per-frame path reads from behaves as a byte queue;
* the host HTTP upgrade (handshake.cpp) equals oracle/ws_handshake.py on
  generated requests.
Streams mix every length class (7-bit, 16-bit and 64-bit, minimal or not),
any RSV / opcode, masked and unmasked frames and a garbage tail."""
import ctypes

import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import gev_amd
from gev_amd import _abi
from oracle import ref
from oracle import ws_oracle as wo

SETTINGS = settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@st.composite
def frame(draw):
    L = draw(st.one_of(st.integers(0, 200), st.sampled_from([125, 126, 127, 300, 1000])))
    forms = [f for f in (7, 16, 64) if (f == 7 and L <= 125) or (f == 16 and L <= 0xFFFF) or f == 64]
    len_form = draw(st.one_of(st.none(), st.sampled_from(forms)))
    return wo.encode_frame(draw(st.binary(min_size=L, max_size=L)), draw(st.integers(0, 15)), draw(st.booleans()),
                           draw(st.integers(0, 7)), draw(st.booleans()), draw(st.binary(min_size=4, max_size=4)),
                           len_form)


streams = st.builds(lambda fs, tail: b"".join(fs) + tail, st.lists(frame(), max_size=12),
                    st.binary(max_size=24))


def _c_decode(streams_):
    arena = np.frombuffer(b"".join(streams_) or b"\0", np.uint8).copy()
    lens = np.array([len(s) for s in streams_])
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]) if len(lens) else np.zeros(0, np.int64)
    return ref.decode_batch(arena, offs, lens)


@SETTINGS
@given(st.lists(streams, min_size=1, max_size=4))
def test_python_and_c_oracles_agree(ss):
    r = _c_decode(ss)
    k = 0
    for ci, s in enumerate(ss):
        res = wo.decode_stream(s)
        assert int(r["conn_nframes"][ci]) == len(res.frames)
        assert int(r["conn_consumed"][ci]) == res.consumed
        assert int(r["conn_status"][ci]) == res.status
        for fr in res.frames:
            f = r["frames"][k]
            assert f.tobytes()[:16] == fr.header.pack()
            o = int(f["payload_off"])
            assert r["payload"][o:o + fr.header.length].tobytes() == fr.payload
            k += 1


@SETTINGS
@given(streams, st.data())
def test_prefix_decodes_to_a_prefix_of_the_frames(s, data):
    cut = data.draw(st.integers(0, len(s)))
    full, part = wo.decode_stream(s), wo.decode_stream(s[:cut])
    assert part.consumed <= cut
    assert len(part.frames) <= len(full.frames)
    for a, b in zip(part.frames, full.frames):
        assert a.header.pack() == b.header.pack() and a.payload == b.payload
    # the leading frames of the full decode that end inside the prefix AND
    # start at least 6 bytes before its end are emitted (read.go:20-23: any
    # header needs 6 readable bytes, even a 2-byte empty frame; Appendix A P1),
    # unless the prefix's own parse stopped on an error first
    start, inside = 0, 0
    for fr in full.frames:
        end = start + fr.header_len + fr.header.length
        if end > cut or cut - start < 6:
            break
        inside += 1
        start = end
    if part.status == wo.OK:
        assert len(part.frames) == inside


def _parse_ring(a: bytes, b: bytes):
    h = _abi.Header()
    hl = ctypes.c_uint32(0)
    ba = (ctypes.c_uint8 * max(len(a), 1)).from_buffer_copy(a or b"\0")
    bb = (ctypes.c_uint8 * max(len(b), 1)).from_buffer_copy(b or b"\0")
    stt = gev_amd.lib.gevws_parse_header_ring(ba if a else None, len(a), bb if b else None, len(b), ctypes.byref(h),
                                              ctypes.byref(hl))
    return stt, h, hl.value


@SETTINGS
@given(st.one_of(frame(), st.binary(max_size=20)), st.data())
def test_parse_header_ring_any_wrap_equals_oracle(buf, data):
    head = buf[:20]
    split = data.draw(st.integers(0, len(head)))
    stt, h, hl = _parse_ring(head[:split], head[split:])
    wst, wh, whl = wo.read_header(head, 0, len(head))
    assert stt == wst
    if stt == wo.OK:
        assert bytes(h) == wh.pack() and hl == whl


@SETTINGS
@given(st.binary(max_size=300), st.binary(min_size=4, max_size=4), st.integers(0, 1 << 20))
def test_host_cipher_equals_bytewise(payload, mask, offset):
    got = (ctypes.c_uint8 * max(len(payload), 1)).from_buffer_copy(payload or b"\0")
    m = (ctypes.c_uint8 * 4).from_buffer_copy(mask)
    gev_amd.lib.gevws_cipher(got, len(payload), m, offset)
    want = bytearray(payload)
    wo.cipher_bytewise(want, mask, offset)
    assert bytes(got)[:len(payload)] == bytes(want)


@SETTINGS
@given(st.integers(1, 64),
       st.lists(st.one_of(st.binary(max_size=100), st.integers(0, 120)), max_size=40))
def test_ring_matches_a_byte_queue(size, ops):
    """The host ring (ringbuffer.RingBuffer as read.go:20,27,63 and
    protocol.go:47-60 use it: Write grows, Retrieve past the end empties) holds
    exactly the bytes written and not yet retrieved, split over at most two
    segments, under any interleaving of writes and retrieves."""
    r, model = gev_amd.RingBuffer(size), bytearray()
    for op in ops:
        if isinstance(op, bytes):
            assert r.write(op) == len(op)
            model += op
        else:
            r.retrieve(op)
            del model[:op]
        a, b = r.peek_all()
        assert a + b == bytes(model)
        assert r.length() == len(model) <= r.capacity()
        assert r.is_empty() == (not model)


_hdr_names = st.sampled_from([b"Host", b"Upgrade", b"Connection", b"Sec-WebSocket-Version", b"Sec-WebSocket-Key",
                              b"Sec-WebSocket-Protocol", b"Sec-WebSocket-Extensions", b"Origin", b"X"])
_hdr_values = st.one_of(st.sampled_from([b"websocket", b"Upgrade", b"13", b"dGhlIHNhbXBsZSBub25jZQ==", b"chat, superchat",
                                         b"permessage-deflate; client_max_window_bits", b""]),
                        st.binary(max_size=40).filter(lambda v: b"\r" not in v and b"\n" not in v))


@SETTINGS
@given(st.lists(st.tuples(_hdr_names, st.sampled_from([b": ", b":", b" :\t"]), _hdr_values), max_size=9),
       st.sampled_from([b"GET", b"PUT", b"get"]), st.sampled_from([b"HTTP/1.1", b"HTTP/1.0", b"HTTP/2.0", b"HTTP/1.1x"]),
       st.binary(max_size=8), st.data())
def test_handshake_equals_oracle(lines, method, proto, tail, data):
    """Upgrader.Upgrade (ws.go:158-343) in the host C++ (handshake.cpp) equals
    oracle/ws_handshake.py byte for byte -- response, status, reason, chosen
    protocol / extensions and bytes consumed -- on generated requests (header
    names in any order, separators, values of arbitrary bytes), with the
    request wrapped round the ring at any point."""
    from tests.test_handshake import _both
    req = method + b" / " + proto + b"\r\n" + b"".join(k + s + v + b"\r\n" for k, s, v in lines) + b"\r\n"
    wrap = data.draw(st.one_of(st.none(), st.integers(1, len(req) + len(tail) - 1)))
    _both(req + tail, wrap_at=wrap)
