"""Shared test helpers: run the HIP decode through the C ABI on host-built
batches and compare it with the oracle, field by field and byte by byte."""
from __future__ import annotations

import numpy as np

from oracle import ref
from oracle import ws_oracle as wo


def gpu_decode(engine, arena: bytes | np.ndarray, conns: np.ndarray, **kw):
    import torch
    import gev_amd
    a = np.frombuffer(arena, np.uint8) if isinstance(arena, (bytes, bytearray)) else arena
    dev = torch.device("cuda", engine.device)
    d_in = torch.zeros(a.size + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    if a.size:
        d_in[: a.size] = torch.from_numpy(a.copy()).to(dev)
    conns = np.ascontiguousarray(conns, dtype=np.int64).reshape(-1, 2)
    d_conns = torch.from_numpy(conns.copy()).to(dev) if conns.shape[0] else torch.zeros((1, 2), dtype=torch.int64,
                                                                                         device=dev)
    out = engine.decode(d_in, a.size, d_conns, conns.shape[0], **kw)
    return out


def host_result(out):
    s = out.summary_host()
    return dict(summary=s, frames=out.frames_host(), conn_out=out.conn_out_host(), payload=out.payload_host())


def check_against_oracle(got: dict, a: np.ndarray, conns: np.ndarray, tag: str = "") -> None:
    """A decode's host-side results (host_result) == the C oracle's on the
    same input, bit-exact, incl. the zeroed pad bytes."""
    conns = np.ascontiguousarray(conns, dtype=np.int64).reshape(-1, 2)
    want = ref.decode_batch(a, conns[:, 0], conns[:, 1])
    s = got["summary"]
    assert int(s["status"]) == 0, tag
    assert int(s["frames"]) == want["frames"].shape[0], tag
    assert int(s["payload_bytes"]) == want["total_payload"], tag
    co = got["conn_out"]
    assert np.array_equal(co["nframes"], want["conn_nframes"]), tag
    assert np.array_equal(co["consumed"], want["conn_consumed"]), tag
    assert np.array_equal(co["status"], want["conn_status"]), tag
    assert np.array_equal(co["first_frame"], want["conn_first"]), tag
    assert int(s["errors"]) == int((want["conn_status"] < 0).sum()), tag
    assert int(s["payload_len"]) == int(want["frames"]["length"].sum()), tag
    assert got["frames"].tobytes() == want["frames"].tobytes(), tag
    assert int(s["run_frames"]) == oracle_run_frames(want, conns), tag
    assert np.array_equal(got["payload"], want["payload"]), tag


def assert_matches_oracle(engine, arena: bytes | np.ndarray, conns: np.ndarray, tag: str = ""):
    """GPU decode == C oracle decode, bit-exact, incl. the zeroed pad bytes."""
    a = np.frombuffer(arena, np.uint8).copy() if isinstance(arena, (bytes, bytearray)) else arena
    conns = np.ascontiguousarray(conns, dtype=np.int64).reshape(-1, 2)
    got = host_result(gpu_decode(engine, a, conns))
    check_against_oracle(got, a, conns, tag)
    return got


def random_batch(rng, n_conns: int, max_len: int = 300, frames=(1, 6)):
    """n_conns random streams (random_stream) packed back to back: (arena, conns)."""
    ss = [random_stream(rng, int(rng.integers(*frames)), max_len=max_len) for _ in range(n_conns)]
    arena = b"".join(ss)
    lens = np.array([len(s) for s in ss], np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    return np.frombuffer(arena, np.uint8).copy(), np.stack([offs, lens], 1)


def post_and_wait(engine, flag, a: np.ndarray, conns: np.ndarray, timeout: float = 5.0):
    """gevws_decode_batch_post of one live pass (inputs resident first: a post
    is not stream-ordered behind torch's copies), then a wait for its number
    in the completion word at flag.host[64:68]; returns its host-side
    results and the device tensors it used."""
    import time
    import torch
    import gev_amd
    dev = torch.device("cuda", engine.device)
    d_in = torch.zeros(a.size + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    if a.size:
        d_in[: a.size] = torch.from_numpy(a).to(dev)
    n = conns.shape[0]
    d_conns = torch.from_numpy(np.ascontiguousarray(conns)).to(dev) if n else torch.zeros((1, 2), dtype=torch.int64,
                                                                                           device=dev)
    max_frames = a.size // 2 + 1
    payload_cap = a.size + 16 * min(max_frames, a.size // 64 + 64) + 64
    out = engine.alloc_batch(n, max_frames, payload_cap)
    # (torch's stream only: a device-wide synchronize would wait for a
    # resident service instance's life to end)
    torch.cuda.current_stream(dev).synchronize()
    engine.decode_post(d_in, a.size, d_conns, n, out, max_frames, payload_cap)
    seq = engine.completion_seq
    assert seq > 0
    word = flag.host[64:68].view(np.uint32)
    t0 = time.monotonic()
    while int(word[0]) != seq:
        assert time.monotonic() - t0 < timeout, f"pass {seq} never signalled (word {int(word[0])})"
    # the outputs are read on torch's stream, beside a resident instance
    return host_result(out), (d_in, d_conns, out)


def oracle_run_frames(want, conns) -> int:
    """summary.run_frames from the oracle's records: frames whose size (h + L)
    equals the size of the frame before them on the same connection."""
    fr = want["frames"]
    n = 0
    for c in range(conns.shape[0]):
        f0, k = int(want["conn_first"][c]), int(want["conn_nframes"][c])
        prev_end, prev = int(conns[c, 0]), None
        for i in range(f0, f0 + k):
            end = int(fr["src_off"][i]) + int(fr["length"][i])
            size = end - prev_end
            n += size == prev
            prev, prev_end = size, end
    return n


def random_stream(rng, n_frames: int, max_len: int = 3072, tail: bool = True) -> bytes:
    s = b""
    for _ in range(n_frames):
        L = int(rng.integers(0, max_len + 1))
        forms = [f for f in (7, 16, 64) if (f != 7 or L <= 125) and (f != 16 or L <= 0xFFFF)]
        form = None if rng.random() < 0.7 else int(rng.choice(forms))
        s += wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), int(rng.integers(0, 16)),
                             bool(rng.random() < 0.8), int(rng.integers(0, 8)) if rng.random() < .1 else 0,
                             bool(rng.random() < 0.85), bytes(rng.integers(0, 256, 4, dtype=np.uint8)), form)
    if tail and rng.random() < 0.7:
        t = wo.encode_frame(bytes(rng.integers(0, 256, 200, dtype=np.uint8)), 2, True, 0, True, b"\x01\x02\x03\x04")
        s += t[: int(rng.integers(1, len(t)))]
    return s


def pack_streams(streams):
    arena = b"".join(streams)
    lens = np.array([len(s) for s in streams], np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64) if len(streams) else np.zeros(0, np.int64)
    return arena, np.stack([offs, lens], axis=1) if len(streams) else np.zeros((0, 2), np.int64)
