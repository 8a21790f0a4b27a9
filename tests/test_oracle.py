"""Oracle pinning (CPU): the restatements in oracle/ against RFC 6455 §5.7
known-answer frames, the Go word-loop vs bytewise definition of ws.Cipher
(cipher.go:14-53), the decode-semantics contract of SURVEY.md Appendix A, and
the committed golden vectors.  Python oracle and C oracle must agree."""
import os

import numpy as np
import pytest

from oracle import ref
from oracle import ws_oracle as wo


# --------------------------------------------------------------------------- RFC KATs
@pytest.mark.parametrize("wire,fin,op,masked,mask,payload", wo.RFC6455_KATS)
def test_rfc6455_kat_python(wire, fin, op, masked, mask, payload):
    # short KATs (< 6 bytes) decode only with more bytes buffered behind them (read.go:20-23)
    st, fr = wo.unpacket(wire + b"\x00" * 6)
    assert st == wo.OK
    h = fr.header
    assert (h.fin, h.opcode, h.masked, h.length) == (fin, op, masked, len(payload))
    assert h.mask == (mask if masked else b"\x00" * 4)
    assert fr.payload == payload
    assert fr.header_len + h.length == len(wire)


@pytest.mark.parametrize("wire,fin,op,masked,length,hlen", wo.RFC6455_HEADER_KATS)
def test_rfc6455_header_kats(wire, fin, op, masked, length, hlen):
    buf = wire + bytes(length)
    st, h, hl = wo.read_header(buf)
    assert st == wo.OK and (h.fin, h.opcode, h.masked, h.length, hl) == (fin, op, masked, length, hlen)
    # the encoder (write.go:48-84 shape) reproduces the KAT header bytes
    assert wo.write_header(fin, 0, op, length, masked) == wire


def test_rfc6455_kat_c_oracle():
    arena = b"".join(k[0] for k in wo.RFC6455_KATS)
    r = ref.decode_batch(np.frombuffer(arena, np.uint8).copy(), np.array([0]), np.array([len(arena)]))
    assert len(r["frames"]) == len(wo.RFC6455_KATS)
    for f, k in zip(r["frames"], wo.RFC6455_KATS):
        L = int(f["length"])
        o = int(f["payload_off"])
        assert r["payload"][o:o + L].tobytes() == k[5]
        assert bool(f["fin"]) == k[1] and f["opcode"] == k[2] and bool(f["masked"]) == k[3]


# --------------------------------------------------------------------------- cipher
def test_cipher_wordloop_equals_bytewise_exhaustive():
    """cipher.go's head/tail/u64 split equals p[i] ^= mask[(off+i)%4] for all
    lengths 0-79 and offsets 0-8."""
    rng = np.random.default_rng(1)
    for n in range(80):
        for off in range(9):
            p = bytes(rng.integers(0, 256, n, dtype=np.uint8))
            mask = bytes(rng.integers(0, 256, 4, dtype=np.uint8))
            a, b = bytearray(p), bytearray(p)
            wo.cipher(a, mask, off)
            wo.cipher_bytewise(b, mask, off)
            assert a == b, (n, off)
            c = np.frombuffer(p, np.uint8).copy()
            ref.cipher(c, mask, off)
            assert c.tobytes() == bytes(b), (n, off)
            assert wo.cipher_np(np.frombuffer(p, np.uint8), mask, off).tobytes() == bytes(b)


def test_cipher_involution_and_composition():
    rng = np.random.default_rng(2)
    for _ in range(50):
        n = int(rng.integers(0, 4000))
        k = int(rng.integers(0, n + 1))
        p = bytes(rng.integers(0, 256, n, dtype=np.uint8))
        mask = bytes(rng.integers(0, 256, 4, dtype=np.uint8))
        a = np.frombuffer(p, np.uint8).copy()
        ref.cipher(a, mask, 0)
        b = a.copy()
        ref.cipher(b, mask, 0)
        assert b.tobytes() == p  # involution
        # Cipher(a||b, k, 0) == Cipher(a, k, 0) || Cipher(b, k, len a)
        x = np.frombuffer(p, np.uint8).copy()
        ref.cipher(x[:k], mask, 0)
        ref.cipher(x[k:], mask, k)
        assert x.tobytes() == a.tobytes()


# --------------------------------------------------------------------------- Appendix A contract
def _mk(payload, op=wo.OP_BINARY, masked=True, mask=b"\x11\x22\x33\x44", **kw):
    return wo.encode_frame(payload, op, kw.pop("fin", True), kw.pop("rsv", 0), masked, mask, kw.pop("len_form", None))


def test_p1_less_than_six_bytes_is_need_more():
    for s in (_mk(b"", masked=False), _mk(b"abc", masked=False)):  # complete 2- and 5-byte frames
        assert len(s) < 6
        assert wo.unpacket(s)[0] == wo.NEED_MORE
    # with one more byte of anything after it, the 5-byte frame decodes
    st, fr = wo.unpacket(_mk(b"abc", masked=False) + b"\x00")
    assert st == wo.OK and fr.payload == b"abc"


def test_p2_payload_incomplete_consumes_nothing():
    s = _mk(bytes(range(50)))
    for cut in range(6, len(s)):
        assert wo.unpacket(s[:cut])[0] == wo.NEED_MORE
    assert wo.decode_stream(s[:-1]).consumed == 0


def test_p3_zero_length_and_p4_unmasked():
    s = _mk(b"") + _mk(b"plain", masked=False) + _mk(b"x" * 10)
    res = wo.decode_stream(s)
    assert [f.payload for f in res.frames] == [b"", b"plain", b"x" * 10]
    assert res.consumed == len(s)


def test_p5_no_validation_and_nonminimal_lengths():
    s = (_mk(b"a" * 5, op=0x3, rsv=7) + _mk(b"b" * 5, op=0xB, len_form=16)
         + _mk(b"c" * 200, op=wo.OP_PING, len_form=64) + _mk(b"d" * 7, op=wo.OP_CLOSE, fin=False))
    res = wo.decode_stream(s)
    assert [(f.header.opcode, f.header.rsv, f.header_len, f.header.fin) for f in res.frames] == [
        (3, 7, 6, True), (0xB, 0, 8, True), (wo.OP_PING, 0, 14, True), (wo.OP_CLOSE, 0, 6, False)]


def test_p7_mask_phase_restarts_per_frame():
    m = b"\x01\x02\x03\x04"
    s = _mk(b"\x00" * 3, mask=m) + _mk(b"\x00" * 5, mask=m)
    assert [f.payload for f in wo.decode_stream(s).frames] == [b"\x00" * 3, b"\x00" * 5]
    raw = s[6:9]
    assert raw == bytes([1, 2, 3])  # the second frame's key starts again at mask[0]


def test_p9_len_msb_poisons():
    bad = bytes([0x82, 0xFF, 0x80, 0, 0, 0, 0, 0, 0, 1, 1, 2, 3, 4, 9])
    assert wo.unpacket(bad)[0] == wo.ERR_LEN_MSB
    res = wo.decode_stream(_mk(b"ok") + bad + _mk(b"never"))
    assert len(res.frames) == 1 and res.status == wo.ERR_LEN_MSB


def test_header_length_classes():
    for L, masked, h in [(0, True, 6), (125, True, 6), (126, True, 8), (65535, True, 8), (65536, True, 14),
                         (0, False, 2), (125, False, 2), (126, False, 4), (65535, False, 4), (65536, False, 10)]:
        s = _mk(bytes(L), masked=masked) + b"\x00" * 6
        st, hdr, hl = wo.read_header(s)
        assert st == wo.OK and hl == h and hdr.length == L


def test_header_pack_is_go_layout():
    h = wo.Header(True, 5, 9, True, b"\x01\x02\x03\x04", 0x0102030405060708)
    b = h.pack()
    assert len(b) == 16 and b[:8] == bytes([1, 5, 9, 1, 1, 2, 3, 4])
    assert int.from_bytes(b[8:], "little") == 0x0102030405060708
    assert wo.Header.unpack(b) == h


# --------------------------------------------------------------------------- golden vectors
def _decode_cases(golden):
    return {k: v for k, v in golden.items() if k != "encode"}


def test_python_oracle_reproduces_golden(golden):
    for name, g in _decode_cases(golden).items():
        arena = g["in"].tobytes()
        k = 0
        poff = 0
        for ci, (off, ln) in enumerate(g["conns"]):
            res = wo.decode_stream(arena[off:off + ln])
            assert (len(res.frames), res.consumed, res.status) == tuple(g["conn_res"][ci]), name
            for fr in res.frames:
                assert fr.header.pack() == g["hdr"][k].tobytes()
                assert int(off) + fr.stream_pos + fr.header_len == int(g["src_off"][k])
                L = int(g["payload_len"][k])
                assert fr.payload == g["payload"][poff:poff + L].tobytes()
                poff += L
                k += 1
        assert k == g["hdr"].shape[0]


def test_c_oracle_reproduces_golden(golden):
    for name, g in _decode_cases(golden).items():
        r = ref.decode_batch(g["in"].copy(), g["conns"][:, 0], g["conns"][:, 1])
        assert np.array_equal(r["conn_nframes"], g["conn_res"][:, 0]), name
        assert np.array_equal(r["conn_consumed"], g["conn_res"][:, 1]), name
        assert np.array_equal(r["conn_status"], g["conn_res"][:, 2]), name
        f = r["frames"]
        assert f.shape[0] == g["hdr"].shape[0]
        assert np.array_equal(f.view(np.uint8).reshape(-1, 32)[:, :16], g["hdr"]), name
        assert np.array_equal(f["src_off"], g["src_off"]), name
        got = b"".join(r["payload"][int(o):int(o) + int(L)].tobytes() for o, L in zip(f["payload_off"], f["length"]))
        assert got == g["payload"].tobytes(), name
        # pad bytes of the 16-byte-aligned arena are zero (make([]byte) zero-fill)
        mask = np.ones(r["payload"].shape[0], bool)
        for o, L in zip(f["payload_off"], f["length"]):
            mask[int(o):int(o) + int(L)] = False
        assert not r["payload"][mask].any()


def test_golden_fixture_generator_is_deterministic(tmp_path):
    import importlib.util
    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location("mg", os.path.join(here, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    mg.OUT = str(tmp_path / "g.npz")
    mg.build()
    a = np.load(mg.OUT)
    b = np.load(os.path.join(here, "golden", "ws_golden.npz"))
    assert sorted(a.files) == sorted(b.files)
    for k in a.files:
        assert np.array_equal(a[k], b[k]), k


def test_python_and_c_oracle_agree_random():
    rng = np.random.default_rng(7)
    streams = []
    for _ in range(20):
        s = b""
        for _ in range(int(rng.integers(0, 30))):
            L = int(rng.integers(0, 3000))
            s += wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), int(rng.integers(0, 16)),
                                 bool(rng.random() < .7), int(rng.integers(0, 8)), bool(rng.random() < .8),
                                 bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
        s += bytes(rng.integers(0, 256, int(rng.integers(0, 20)), dtype=np.uint8))
        streams.append(s)
    arena = np.frombuffer(b"".join(streams), np.uint8).copy()
    lens = np.array([len(s) for s in streams])
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    r = ref.decode_batch(arena, offs, lens)
    k = 0
    for ci, s in enumerate(streams):
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


def test_python_and_c_oracle_agree_on_noise():
    """Pure random bytes (the GPU garbage-stream test's input class): headers
    parsed from noise, ErrHeaderLengthMSB, incomplete tails -- both oracles
    agree frame by frame."""
    rng = np.random.default_rng(8)
    streams = [bytes(rng.integers(0, 256, int(rng.integers(0, 2000)), dtype=np.uint8)) for _ in range(60)]
    arena = np.frombuffer(b"".join(streams), np.uint8).copy()
    lens = np.array([len(s) for s in streams])
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    r = ref.decode_batch(arena, offs, lens)
    k = 0
    statuses = set()
    for ci, s in enumerate(streams):
        res = wo.decode_stream(s)
        statuses.add(res.status)
        assert int(r["conn_nframes"][ci]) == len(res.frames)
        assert int(r["conn_consumed"][ci]) == res.consumed
        assert int(r["conn_status"][ci]) == res.status
        for fr in res.frames:
            f = r["frames"][k]
            assert f.tobytes()[:16] == fr.header.pack()
            o = int(f["payload_off"])
            assert r["payload"][o:o + fr.header.length].tobytes() == fr.payload
            k += 1
    assert k > 0 and len(statuses) > 1  # noise produced frames and more than one outcome


# --------------------------------------------------------------------------- outbound encode
def _h(**kw):
    return wo.Header(**kw)


def test_write_header_rfc_kats():
    assert wo.write_header_go(_h(fin=True, opcode=1, length=5)) == bytes.fromhex("8105")
    assert wo.write_header_go(_h(fin=True, opcode=2, length=256)) == bytes.fromhex("827e0100")
    assert wo.write_header_go(_h(fin=True, opcode=2, length=65536)) == bytes.fromhex("827f0000000000010000")
    assert wo.write_header_go(_h(fin=True, opcode=1, masked=True, mask=bytes.fromhex("37fa213d"),
                                 length=5)) == bytes.fromhex("818537fa213d")
    h, p = wo.new_frame(wo.OP_TEXT, True, b"Hello")
    assert wo.frame_to_bytes(h, p) == bytes.fromhex("810548656c6c6f")  # RFC 6455 §5.7


def test_write_header_go_byte_arithmetic():
    assert wo.write_header_go(_h(rsv=8, opcode=1, length=0))[0] == 0x81          # Rsv<<4 overflows into FIN
    assert wo.write_header_go(_h(rsv=0x13, opcode=0x1F, length=0))[0] == 0x3F    # (0x130 & 0xff) | 0x1f
    assert wo.write_header_go(_h(length=-1)) == bytes([0x00, 0xFF])              # byte(-1), 2-byte form
    assert wo.write_header_go(_h(length=-1, masked=True, mask=b"abcd")) == bytes([0x00, 0xFF]) + b"abcd"
    assert wo.write_header_go(_h(length=(1 << 63) - 1))[1:] == bytes([127, 0x7F] + [0xFF] * 7)


def test_write_header_python_equals_c():
    rng = np.random.default_rng(31)
    for _ in range(3000):
        h = wo.Header(bool(rng.random() < .5), int(rng.integers(0, 256)), int(rng.integers(0, 256)),
                      bool(rng.random() < .5), bytes(rng.integers(0, 256, 4, dtype=np.uint8)),
                      int(rng.choice([int(rng.integers(-(1 << 40), 1 << 40)), int(rng.integers(0, 200)),
                                      int(rng.integers(60000, 70000)), (1 << 63) - 1, -(1 << 63)])))
        assert ref.write_header(h.pack()) == wo.write_header_go(h)


def test_encode_golden_c_and_python(golden):
    g = golden["encode"]
    offs = np.concatenate([[0], np.cumsum(g["payload_len"])[:-1]])
    fr = np.zeros(g["hdr"].shape[0], ref.OUT_FRAME_DTYPE)
    fr.view(np.uint8).reshape(-1, 32)[:, :16] = g["hdr"]
    fr["payload_off"] = offs
    fr["payload_len"] = g["payload_len"]
    wire, off = ref.encode_batch(fr, g["payload"])
    assert np.array_equal(wire, g["wire"]) and np.array_equal(off.astype(np.int64), g["out_off"])
    py = b"".join(wo.frame_to_bytes(wo.Header.unpack(h.tobytes()), g["payload"][o:o + L].tobytes())
                  for h, o, L in zip(g["hdr"], offs, g["payload_len"]))
    assert py == g["wire"].tobytes()


def test_encode_decode_round_trip():
    """decode(FrameToBytes(NewBinaryFrame(p))) == p -- the echo server's reply
    (benchmarks/websocket/server.go:22-29) read back by a client."""
    rng = np.random.default_rng(32)
    for L in (0, 1, 125, 126, 65535, 65536, 70001):
        p = bytes(rng.integers(0, 256, L, dtype=np.uint8))
        h, _ = wo.new_frame(wo.OP_BINARY, True, p)
        res = wo.decode_stream(wo.frame_to_bytes(h, p) + b"\x00" * 6)
        assert res.frames[0].payload == p and res.frames[0].header.opcode == wo.OP_BINARY


# --------------------------------------------------------------------------- control-frame dispatch
def test_dispatch_oracle_reference_behaviour():
    H = lambda op, L: wo.Header(fin=True, opcode=op, masked=True, mask=b"abcd", length=L)  # noqa: E731
    # ping -> pong, pong -> PING (util.go:49-56, the reference's quirk)
    assert wo.on_message(H(9, 2), b"hi", 0) == (bytes([0x8A, 2]) + b"hi", False)
    assert wo.on_message(H(10, 2), b"hi", 0) == (bytes([0x89, 2]) + b"hi", False)
    # empty close -> bare close header + ShutdownWrite (util.go:28-33, wrap.go:56)
    assert wo.on_message(H(8, 0), b"", 0) == (bytes([0x88, 0x00]), True)
    # valid close echoes code + reason; reason cropped to 123 bytes (frame.go:251-259)
    r, sd = wo.on_message(H(8, 2 + 200), (1000).to_bytes(2, "big") + b"x" * 200, 0)
    assert sd and r[:4] == bytes([0x88, 125, 0x03, 0xE8]) and len(r) == 2 + 125
    # code/UTF-8 checks in util.go:65-85 order
    for code, msg in [(999, wo.ERR_NOT_IN_USE), (1005, wo.ERR_APP_LEVEL), (1004, wo.ERR_NO_MEANING),
                      (1012, wo.ERR_UNKNOWN)]:
        r, _ = wo.on_message(H(8, 3), code.to_bytes(2, "big") + b"a", 0)
        assert r == bytes([0x88, 2 + len(msg), 0x03, 0xEA]) + msg
    r, _ = wo.on_message(H(8, 3), (3000).to_bytes(2, "big") + b"\xff", 0)
    assert r.endswith(wo.ERR_INVALID_UTF8)
    # 1-byte close payload: ParseCloseFrameData -> code 0 -> not in use
    assert wo.on_message(H(8, 1), b"\x03", 0)[0].endswith(wo.ERR_NOT_IN_USE)
    # reserved control opcodes: nothing; data: the policy; empty data: nothing (wrap.go:72)
    assert wo.on_message(H(0xB, 1), b"r", 1) == (None, False)
    assert wo.on_message(H(1, 3), b"abc", wo.HANDLER_ECHO_BINARY)[0] == bytes([0x82, 3]) + b"abc"
    assert wo.on_message(H(0, 3), b"abc", wo.HANDLER_ECHO_TEXT)[0] == bytes([0x81, 3]) + b"abc"
    assert wo.on_message(H(2, 0), b"", wo.HANDLER_ECHO_BINARY) == (None, False)
    assert wo.on_message(H(2, 3), b"abc", wo.HANDLER_NONE) == (None, False)


def test_utf8_validation_is_strict():
    ok = ["", "abc", "héllo", "日本", "\U0001F600", "﻿"]
    bad = [b"\xff", b"\xc0\xaf", b"\xed\xa0\x80", b"\xe2\x82", b"\xf4\x90\x80\x80", b"\xe0\x80\xaf", b"a\x80"]
    assert all(wo.utf8_valid(x.encode()) for x in ok)
    assert not any(wo.utf8_valid(b) for b in bad)


@pytest.mark.parametrize("alloc", ["fresh", "cache_hot"])
@pytest.mark.parametrize("vectorized", [False, True])
def test_cpu_baseline_pipeline_allocation_modes(alloc, vectorized):
    """The CPU baseline's per-frame pipeline (oracle/ws_ref.c, bench.py
    cpu_baseline) in both allocation modes and both builds processes whole
    passes over the batch: on one thread its payload bytes and frames are
    exact multiples of the batch's own (each of 3 threads repeats its own
    share of the connections)."""
    rng = np.random.default_rng(7)
    streams = [b"".join(wo.encode_frame(bytes(rng.integers(0, 256, int(L), dtype=np.uint8)), 2, True, 0, True,
                                        b"\x01\x02\x03\x04") for L in rng.integers(0, 70000, 6))
               for _ in range(5)]
    arena = np.frombuffer(b"".join(streams) + bytes(64), np.uint8).copy()
    lens = np.array([len(s) for s in streams], np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    want = ref.decode_batch(arena[:-64], offs, lens)
    per_pass_bytes, per_pass_frames = int(want["frames"]["length"].sum()), want["frames"].shape[0]
    for threads in (1, 3):
        secs, pb, nf = ref.bench_pipeline(arena, offs, lens, threads=threads, min_seconds=0.05,
                                          vectorized=vectorized, alloc=alloc)
        assert secs > 0 and nf > 0 and pb > 0
        if threads == 1:
            assert pb * per_pass_frames == nf * per_pass_bytes
    assert ref.fresh_arena_bytes() >= 64 << 20
