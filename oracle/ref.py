"""ctypes binding for oracle/libwsref.so (the C restatement).

TEST INFRASTRUCTURE ONLY -- see ws_oracle.py header.  Used by tests/ (as the
checker at medium sizes), __graft_entry__.smoke() and bench.py's cpu_baseline.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_VEC = None

FRAME_DTYPE = np.dtype([("fin", "u1"), ("rsv", "u1"), ("opcode", "u1"), ("masked", "u1"),
                        ("mask", "u1", (4,)), ("length", "<i8"),
                        ("payload_off", "<u8"), ("src_off", "<u8")])
assert FRAME_DTYPE.itemsize == 32
OUT_FRAME_DTYPE = np.dtype([("fin", "u1"), ("rsv", "u1"), ("opcode", "u1"), ("masked", "u1"),
                            ("mask", "u1", (4,)), ("length", "<i8"),
                            ("payload_off", "<u8"), ("payload_len", "<u8")])


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "libwsref.so")


def _load(name: str):
    path = os.path.join(_HERE, name)
    if not os.path.exists(path):
        build()
    return ctypes.CDLL(path)


def vec_lib():
    """The -O3 -mavx2 build of the same restatement (bench pipeline only)."""
    global _VEC
    if _VEC is None:
        L = _load("libwsref_vec.so")
        P = ctypes.c_void_p
        L.wsref_bench_pipeline.argtypes = [P, P, P, ctypes.c_uint32, ctypes.c_int, ctypes.c_double,
                                           P, P, P]
        L.wsref_bench_pipeline.restype = ctypes.c_double
        L.wsref_bench_pipeline_alloc.argtypes = [P, P, P, ctypes.c_uint32, ctypes.c_int, ctypes.c_double,
                                                 ctypes.c_int, ctypes.c_uint64, P, P, P]
        L.wsref_bench_pipeline_alloc.restype = ctypes.c_double
        _VEC = L
    return _VEC


def lib():
    global _LIB
    if _LIB is None:
        L = _load("libwsref.so")
        P = ctypes.c_void_p
        L.wsref_cipher.argtypes = [P, ctypes.c_size_t, P, ctypes.c_size_t]
        L.wsref_cipher.restype = None
        L.wsref_read_header.argtypes = [P, ctypes.c_uint64, P, P]
        L.wsref_read_header.restype = ctypes.c_int
        L.wsref_decode_batch.argtypes = [P, P, P, ctypes.c_uint32, P, ctypes.c_uint64, P,
                                         ctypes.c_uint64, P, P, P, P, P]
        L.wsref_decode_batch.restype = ctypes.c_int64
        L.wsref_write_header.argtypes = [P, P]
        L.wsref_write_header.restype = ctypes.c_uint32
        L.wsref_encode_batch.argtypes = [P, ctypes.c_uint64, P, P, ctypes.c_uint64, P]
        L.wsref_encode_batch.restype = ctypes.c_int64
        L.wsref_bench_pipeline.argtypes = [P, P, P, ctypes.c_uint32, ctypes.c_int, ctypes.c_double,
                                           P, P, P]
        L.wsref_bench_pipeline.restype = ctypes.c_double
        L.wsref_bench_pipeline_alloc.argtypes = [P, P, P, ctypes.c_uint32, ctypes.c_int, ctypes.c_double,
                                                 ctypes.c_int, ctypes.c_uint64, P, P, P]
        L.wsref_bench_pipeline_alloc.restype = ctypes.c_double
        _LIB = L
    return _LIB


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def cipher(buf: np.ndarray, mask: bytes, offset: int = 0) -> None:
    """In-place ws.Cipher word-loop restatement on a uint8 numpy array."""
    m = np.frombuffer(mask, dtype=np.uint8).copy()
    lib().wsref_cipher(_ptr(buf), buf.size, _ptr(m), offset)


def decode_batch(arena: np.ndarray, conn_off: np.ndarray, conn_len: np.ndarray,
                 max_frames: int | None = None, payload_cap: int | None = None):
    """Oracle decode of a batch in the product's output layout.

    Returns dict(frames, payload, conn_first, conn_nframes, conn_status,
    conn_consumed, total_payload) or raises on capacity error."""
    n = conn_off.size
    conn_off = np.ascontiguousarray(conn_off, dtype=np.uint64)
    conn_len = np.ascontiguousarray(conn_len, dtype=np.uint64)
    total_in = int(conn_len.sum()) if n else 0
    if max_frames is None:
        max_frames = total_in // 2 + 1
    if payload_cap is None:
        payload_cap = total_in + 16 * max_frames + 16
    frames = np.zeros(max_frames, dtype=FRAME_DTYPE)
    payload = np.zeros(payload_cap, dtype=np.uint8)
    first = np.zeros(max(n, 1), dtype=np.uint64)
    nfr = np.zeros(max(n, 1), dtype=np.uint32)
    st = np.zeros(max(n, 1), dtype=np.int32)
    cons = np.zeros(max(n, 1), dtype=np.uint64)
    tot = np.zeros(1, dtype=np.uint64)
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    nf = lib().wsref_decode_batch(_ptr(arena), _ptr(conn_off), _ptr(conn_len), n, _ptr(frames),
                                  max_frames, _ptr(payload), payload_cap, _ptr(first), _ptr(nfr),
                                  _ptr(st), _ptr(cons), _ptr(tot))
    if nf < 0:
        raise RuntimeError(f"wsref_decode_batch failed: {nf}")
    tp = int(tot[0])
    return dict(frames=frames[:nf], payload=payload[:tp], conn_first=first[:n],
                conn_nframes=nfr[:n], conn_status=st[:n], conn_consumed=cons[:n],
                total_payload=tp)


ALLOC_FRESH, ALLOC_CACHE_HOT = 0, 1  # ws_ref.c WSREF_ALLOC_*


def llc_slice_bytes() -> int:
    """The last-level cache one CPU sees (cpu0's highest cache index), or 32 MiB."""
    base = "/sys/devices/system/cpu/cpu0/cache"
    best = 0
    try:
        for d in os.listdir(base):
            if not d.startswith("index"):
                continue
            sz = open(os.path.join(base, d, "size")).read().strip()
            mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(sz[-1:], 1)
            best = max(best, int(sz.rstrip("KMG")) * mult)
    except (OSError, ValueError):
        pass
    return best or (32 << 20)


def fresh_arena_bytes() -> int:
    """Per-thread arena of the fresh-allocation mode: twice the LLC one CPU
    sees, at least 64 MiB -- a thread's destinations are never cache-resident."""
    return max(64 << 20, 2 * llc_slice_bytes())


def bench_pipeline(arena: np.ndarray, conn_off: np.ndarray, conn_len: np.ndarray,
                   threads: int = 1, min_seconds: float = 10.0, vectorized: bool = False,
                   alloc: str = "fresh"):
    """Time the reference per-frame pipeline; returns (seconds, payload_bytes, frames).
    vectorized=True times the -O3 -mavx2 build of the same C source.  alloc:
    "fresh" (each frame's zero-filled destination from a per-thread bump arena
    of fresh_arena_bytes(), as Go's make hands out swept memory) or
    "cache_hot" (calloc / free per frame: glibc recycles one warm chunk)."""
    pb = np.zeros(1, dtype=np.uint64)
    nf = np.zeros(1, dtype=np.uint64)
    ck = np.zeros(1, dtype=np.uint64)
    conn_off = np.ascontiguousarray(conn_off, dtype=np.uint64)
    conn_len = np.ascontiguousarray(conn_len, dtype=np.uint64)
    L = vec_lib() if vectorized else lib()
    mode = {"fresh": ALLOC_FRESH, "cache_hot": ALLOC_CACHE_HOT}[alloc]
    secs = L.wsref_bench_pipeline_alloc(_ptr(arena), _ptr(conn_off), _ptr(conn_len), conn_off.size,
                                        threads, min_seconds, mode, fresh_arena_bytes(),
                                        _ptr(pb), _ptr(nf), _ptr(ck))
    if secs < 0:
        raise MemoryError("wsref_bench_pipeline_alloc: arena allocation failed")
    return secs, int(pb[0]), int(nf[0])


def write_header(hdr16: bytes) -> bytes:
    """ws.WriteHeader on a packed 16-byte ws.Header image."""
    h = np.frombuffer(hdr16, np.uint8).copy()
    out = np.zeros(14, np.uint8)
    n = lib().wsref_write_header(_ptr(h), _ptr(out))
    return out[:n].tobytes()


def encode_batch(frames: np.ndarray, payload: np.ndarray):
    """FrameToBytes for every record of `frames` (OUT_FRAME_DTYPE), back to back.
    Returns (wire bytes as uint8 array, out_off)."""
    frames = np.ascontiguousarray(frames)
    cap = int(frames["payload_len"].sum()) + 14 * frames.shape[0] + 16
    out = np.zeros(cap, np.uint8)
    off = np.zeros(max(frames.shape[0], 1), np.uint64)
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    if payload.size == 0:
        payload = np.zeros(1, np.uint8)
    tot = lib().wsref_encode_batch(_ptr(frames), frames.shape[0], _ptr(payload), _ptr(out), cap, _ptr(off))
    if tot < 0:
        raise RuntimeError("wsref_encode_batch failed")
    return out[:tot], off[:frames.shape[0]]
