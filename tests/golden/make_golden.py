"""Generate tests/golden/ws_golden.npz -- golden decode vectors for the hot path.

The reference (Go) cannot run here and holds no vectors for this path
(SURVEY.md §4, §8c), so the expected outputs come from the bytewise Python
restatement oracle/ws_oracle.py, whose arithmetic is pinned by the RFC 6455
§5.7 known-answer frames (included verbatim as case ``rfc_kats``).  Cases
exclude the ringbuffer-dependent rows U1-U3 of SURVEY.md Appendix A except
where the oracle's documented choice is exercised on purpose (``u1_partial``).

Run:  python tests/golden/make_golden.py     (deterministic; seed fixed)
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import ws_oracle as wo  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ws_golden.npz")


def rand_mask(rng):
    return bytes(rng.integers(0, 256, 4, dtype=np.uint8))


def case_rfc_kats(rng):
    return [b"".join(k[0] for k in wo.RFC6455_KATS)]


def case_header_classes(rng):
    s = b""
    for L in (0, 1, 5, 7, 8, 15, 16, 17, 125, 126, 127, 1000, 65535, 65536, 70001):
        for masked in (True, False):
            p = bytes(rng.integers(0, 256, L, dtype=np.uint8))
            s += wo.encode_frame(p, wo.OP_BINARY, True, 0, masked, rand_mask(rng))
    # 6 trailing bytes of an incomplete masked 7-bit frame: NEED_MORE at the end
    s += wo.encode_frame(b"abcdefgh", wo.OP_TEXT, True, 0, True, b"\x01\x02\x03\x04")[:7]
    return [s]


def case_mixed_random(rng, n=300):
    """wsserver_test.go:112-117 shape (masked text, 1-3072 random bytes) mixed
    with every header form, RSV bits, reserved opcodes, FIN=0 and non-minimal
    length encodings (Appendix A P3-P8)."""
    s = b""
    for i in range(n):
        kind = rng.random()
        L = int(rng.integers(1, 3073)) if kind < 0.6 else int(rng.integers(0, 200))
        op = int(rng.choice([0, 1, 2, 3, 7, 8, 9, 10, 11, 15]))
        fin = bool(rng.random() < 0.8)
        rsv = int(rng.integers(0, 8)) if rng.random() < 0.2 else 0
        masked = bool(rng.random() < 0.85)
        forms = [f for f in (7, 16, 64) if (f != 7 or L <= 125) and (f != 16 or L <= 0xFFFF)]
        form = None if rng.random() < 0.7 else int(rng.choice(forms))
        p = bytes(rng.integers(0, 256, L, dtype=np.uint8))
        s += wo.encode_frame(p, op, fin, rsv, masked, rand_mask(rng), form)
    # partial last frame (payload incomplete: Appendix A P2)
    s += wo.encode_frame(bytes(100), wo.OP_BINARY, True, 0, True, rand_mask(rng))[:60]
    return [s]


def case_short_tail(rng):
    # complete unmasked 2..5-byte frames at the end are NOT decoded (< 6 bytes, P1)
    a = wo.encode_frame(b"hello world", wo.OP_TEXT, True, 0, True, b"\xaa\xbb\xcc\xdd")
    return [a + wo.encode_frame(b"", wo.OP_PING, True, 0, False),
            a + wo.encode_frame(b"xyz", wo.OP_TEXT, True, 0, False),
            a + wo.encode_frame(b"xy", wo.OP_TEXT, True, 0, False) + b"\x81"]


def case_poison(rng):
    a = wo.encode_frame(b"before", wo.OP_TEXT, True, 0, True, b"\x10\x20\x30\x40")
    bad = bytes([0x82, 0xFF, 0x80, 0, 0, 0, 0, 0, 0, 5]) + b"\x01\x02\x03\x04" + b"12345"
    tail = wo.encode_frame(b"after", wo.OP_TEXT, True, 0, True, b"\x10\x20\x30\x40")
    return [a + bad + tail]


def case_u1_partial(rng):
    # avail >= 6 but < header length: oracle's documented NEED_MORE choice (U1)
    f = wo.encode_frame(bytes(70000), wo.OP_BINARY, True, 0, True, b"\x01\x02\x03\x04")
    g = wo.encode_frame(bytes(300), wo.OP_BINARY, True, 0, True, b"\x01\x02\x03\x04")
    return [f[:9], f[:13], g[:7], wo.encode_frame(b"ok", wo.OP_TEXT, True, 0, True, b"\x05\x06\x07\x08") + g[:7]]


def case_multi_conn(rng, n_conns=37):
    conns = []
    for c in range(n_conns):
        s = b""
        for _ in range(int(rng.integers(0, 12))):
            L = int(rng.integers(0, 5000))
            s += wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), int(rng.choice([1, 2, 9, 10])),
                                 True, 0, bool(rng.random() < 0.9), rand_mask(rng))
        if rng.random() < 0.5:
            t = wo.encode_frame(bytes(rng.integers(0, 256, 300, dtype=np.uint8)), 2, True, 0, True, rand_mask(rng))
            s += t[: int(rng.integers(1, len(t)))]
        conns.append(s)
    return conns


def encode_case(rng, n=400):
    """ws.FrameToBytes inputs: server replies (NewBinaryFrame/NewTextFrame/
    pong/close) plus hand-built headers exercising Go's byte arithmetic in
    WriteHeader (Rsv > 7, OpCode > 15, negative and boundary lengths, Masked
    without payload masking)."""
    hdrs, pays = [], []
    for i in range(n):
        L = int(rng.choice([0, 1, 2, 5, 125, 126, 127, 1000, 3072]))
        L = min(L, int(rng.integers(0, 3000))) if rng.random() < 0.5 else L
        if i in (7, 100, 333):
            L = (65535, 65536, 70000)[(7, 100, 333).index(i)]
        p = bytes(rng.integers(0, 256, L, dtype=np.uint8)) if L < 4096 else bytes(np.arange(L) % 251)
        if rng.random() < 0.7:
            h, p = wo.new_frame(int(rng.choice([1, 2, 8, 9, 10])), True, p)
        else:
            h = wo.Header(bool(rng.random() < .5), int(rng.integers(0, 256)), int(rng.integers(0, 256)),
                          bool(rng.random() < .5), bytes(rng.integers(0, 256, 4, dtype=np.uint8)),
                          int(rng.choice([len(p), -1, -300, 125, 126, 65535, 65536, (1 << 63) - 1])))
        hdrs.append(h)
        pays.append(p)
    return hdrs, pays


CASES = {
    "rfc_kats": case_rfc_kats,
    "header_classes": case_header_classes,
    "mixed_random": case_mixed_random,
    "short_tail": case_short_tail,
    "poison": case_poison,
    "u1_partial": case_u1_partial,
    "multi_conn": case_multi_conn,
}


def build():
    rng = np.random.default_rng(0x67657600)
    arrays = {}
    for name, fn in CASES.items():
        streams = fn(rng)
        arena = b"".join(streams)
        offs = np.cumsum([0] + [len(s) for s in streams[:-1]]).astype(np.int64)
        conns = np.stack([offs, np.array([len(s) for s in streams], np.int64)], axis=1)
        hdrs, srcs, payloads, conn_res = [], [], [], []
        for ci, s in enumerate(streams):
            res = wo.decode_stream(s)
            for fr in res.frames:
                hdrs.append(np.frombuffer(fr.header.pack(), np.uint8))
                srcs.append(int(offs[ci]) + fr.stream_pos + fr.header_len)
                payloads.append(fr.payload)
            conn_res.append((len(res.frames), res.consumed, res.status))
        arrays[f"{name}/in"] = np.frombuffer(arena, np.uint8)
        arrays[f"{name}/conns"] = conns
        arrays[f"{name}/hdr"] = np.array(hdrs, np.uint8).reshape(-1, 16)
        arrays[f"{name}/src_off"] = np.array(srcs, np.uint64)
        arrays[f"{name}/payload_len"] = np.array([len(p) for p in payloads], np.int64)
        arrays[f"{name}/payload"] = np.frombuffer(b"".join(payloads), np.uint8)
        arrays[f"{name}/conn_res"] = np.array(conn_res, np.int64).reshape(-1, 3)
    hdrs, pays = encode_case(rng)
    arrays["encode/hdr"] = np.array([np.frombuffer(h.pack(), np.uint8) for h in hdrs], np.uint8)
    arrays["encode/payload_len"] = np.array([len(p) for p in pays], np.int64)
    arrays["encode/payload"] = np.frombuffer(b"".join(pays), np.uint8)
    wires = [wo.frame_to_bytes(h, p) for h, p in zip(hdrs, pays)]
    arrays["encode/wire"] = np.frombuffer(b"".join(wires), np.uint8)
    arrays["encode/out_off"] = np.concatenate([[0], np.cumsum([len(x) for x in wires])[:-1]]).astype(np.int64)
    np.savez_compressed(OUT, **arrays)
    return OUT


if __name__ == "__main__":
    p = build()
    print(p, os.path.getsize(p), "bytes")
