"""CPU parity of the per-frame host exports of the boundary (SURVEY.md §8b
items 1-2): gevws_parse_header / gevws_parse_header_ring against the oracle's
ws.VirtualReadHeader restatement (read.go:19-84) and gevws_cipher against the
ws.Cipher restatements (cipher.go:14-53), on the golden fixtures, every
header-length class, every availability 0..16 and random byte windows."""
import ctypes

import numpy as np
import pytest

import gev_amd
from gev_amd import _abi
from oracle import ref
from oracle import ws_oracle as wo

lib = gev_amd.lib


def parse(buf: bytes, avail: int | None = None):
    if avail is None:
        avail = len(buf)
    h = _abi.Header()
    hl = ctypes.c_uint32(77)
    b = (ctypes.c_uint8 * max(len(buf), 1)).from_buffer_copy(buf or b"\0")
    st = lib.gevws_parse_header(b, avail, ctypes.byref(h), ctypes.byref(hl))
    return st, h, hl.value


def parse_ring(a: bytes, b: bytes):
    h = _abi.Header()
    hl = ctypes.c_uint32(77)
    ba = (ctypes.c_uint8 * max(len(a), 1)).from_buffer_copy(a or b"\0")
    bb = (ctypes.c_uint8 * max(len(b), 1)).from_buffer_copy(b or b"\0")
    st = lib.gevws_parse_header_ring(ba if a else None, len(a), bb if b else None, len(b), ctypes.byref(h),
                                     ctypes.byref(hl))
    return st, h, hl.value


def expected_hlen(buf: bytes) -> int:
    if len(buf) < 2:
        return 0
    len7 = buf[1] & 0x7F
    return 2 + (0 if len7 < 126 else (2 if len7 == 126 else 8)) + (4 if buf[1] & 0x80 else 0)


def check_against_oracle(buf: bytes, avail: int):
    st, h, hl = parse(buf, avail)
    wst, wh, whl = wo.read_header(buf, 0, avail)
    assert st == wst, (buf[:16].hex(), avail)
    if st == wo.OK:
        assert bytes(h) == wh.pack(), (buf[:16].hex(), avail)
        assert hl == whl
    elif st == wo.NEED_MORE:
        assert hl == (expected_hlen(buf[:avail]) if avail >= 2 else 0)


def test_parse_header_golden_frame_starts(golden):
    for case, d in golden.items():
        if "conns" not in d:  # encode / dispatch fixtures hold no input streams
            continue
        arena = d["in"].tobytes()
        conns = d["conns"].reshape(-1, 2)
        for off, ln in conns:
            s = arena[int(off):int(off) + int(ln)]
            r = wo.decode_stream(s)
            starts = [f.stream_pos for f in r.frames] + [r.consumed]
            for p in starts:
                for avail in sorted({0, 1, 2, 5, 6, 7, 13, 14, len(s) - p}):
                    if 0 <= avail <= len(s) - p:
                        check_against_oracle(s[p:], avail)


def test_parse_header_every_class_and_availability():
    rng = np.random.default_rng(5)
    for L in (0, 1, 5, 125, 126, 127, 1000, 65535, 65536, 70001, 1 << 40):
        for masked in (False, True):
            forms = [f for f in (7, 16, 64) if (f != 7 or L <= 125) and (f != 16 or L <= 0xFFFF)]
            for form in forms:
                hdr = wo.write_header(True, int(rng.integers(0, 8)), int(rng.integers(0, 16)), L, masked,
                                      bytes(rng.integers(0, 256, 4, dtype=np.uint8)), form)
                buf = hdr + bytes(rng.integers(0, 256, 20, dtype=np.uint8))
                for avail in range(0, len(buf) + 1):
                    check_against_oracle(buf, avail)


def test_parse_header_len_msb_and_random_windows():
    # 64-bit length with the MSB set: ErrHeaderLengthMSB (read.go:71-73)
    buf = bytes([0x82, 0xFF, 0x80, 0, 0, 0, 0, 0, 0, 1, 1, 2, 3, 4])
    st, _, hl = parse(buf)
    assert st == gev_amd.ERR_LEN_MSB and hl == 14
    rng = np.random.default_rng(6)
    for _ in range(20000):
        buf = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        check_against_oracle(buf, int(rng.integers(0, 17)))


def test_parse_header_ring_every_split():
    rng = np.random.default_rng(7)
    for _ in range(300):
        L = int(rng.choice([3, 126, 300, 70000]))
        hdr = wo.write_header(True, 0, 2, L, bool(rng.random() < 0.8), bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
        buf = hdr + bytes(rng.integers(0, 256, int(rng.integers(0, 30)), dtype=np.uint8))
        for k in range(len(buf) + 1):
            st, h, hl = parse_ring(buf[:k], buf[k:])
            st2, h2, hl2 = parse(buf)
            assert (st, hl) == (st2, hl2)
            if st == gev_amd.OK:
                assert bytes(h) == bytes(h2)
    assert parse_ring(b"", b"")[0] == gev_amd.NEED_MORE


def test_parse_header_invalid_arguments():
    h = _abi.Header()
    assert lib.gevws_parse_header(None, 4, ctypes.byref(h), None) == gev_amd.ERR_INVALID
    assert lib.gevws_parse_header(None, 0, None, None) == gev_amd.ERR_INVALID
    assert lib.gevws_parse_header(None, 0, ctypes.byref(h), None) == gev_amd.NEED_MORE


def host_cipher(p: bytes, mask: bytes, offset: int) -> bytes:
    b = (ctypes.c_uint8 * max(len(p), 1)).from_buffer_copy(p or b"\0")
    m = (ctypes.c_uint8 * 4)(*mask)
    lib.gevws_cipher(b, len(p), m, offset)
    return bytes(b)[:len(p)]


def test_host_cipher_exhaustive_small():
    """Every length 0-79 x offset 0-8 against the bytewise
    definition and the C word-loop restatement."""
    rng = np.random.default_rng(8)
    for n in range(80):
        for off in range(9):
            p = bytes(rng.integers(0, 256, n, dtype=np.uint8))
            mask = bytes(rng.integers(0, 256, 4, dtype=np.uint8))
            want = bytearray(p)
            wo.cipher_bytewise(want, mask, off)
            assert host_cipher(p, mask, off) == bytes(want), (n, off)
            c = np.frombuffer(p, np.uint8).copy()
            ref.cipher(c, mask, off)
            assert c.tobytes() == bytes(want)


@pytest.mark.parametrize("n", [1 << 10, 65536 + 13, (1 << 20) + 7])
def test_host_cipher_large_unaligned_involution(n):
    rng = np.random.default_rng(n)
    raw = bytes(rng.integers(0, 256, n + 16, dtype=np.uint8))
    mask = bytes(rng.integers(0, 256, 4, dtype=np.uint8))
    for start in (0, 1, 3, 7):
        p = raw[start:start + n]
        off = int(rng.integers(0, 1000))
        got = host_cipher(p, mask, off)
        assert got == wo.cipher_np(p, mask, off).tobytes()
        assert host_cipher(got, mask, off) == p  # involution
