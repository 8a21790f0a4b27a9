"""Synthetic batch layouts for the BASELINE.json configs.

A layout is a frame-descriptor table (SYNTH_DTYPE: header offset, payload
length, key, first header byte, length form, masked) plus the per-connection
stream table (offset, length) inside one input arena.  The device generator
(gevws_synth_async) writes the frames; nothing of batch size is built on the
host.  Connections are independent byte streams, laid out back to back with no
alignment (frame payloads start at arbitrary byte offsets, as they do in a
ring buffer).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import SYNTH_DTYPE

GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 on uint64 arrays (wrapping arithmetic), same as the device generator."""
    with np.errstate(over="ignore"):
        x = (x + GOLDEN).astype(np.uint64)
        x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)).astype(np.uint64)
        x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)).astype(np.uint64)
        return x ^ (x >> np.uint64(31))


def frame_masks(n: int, seed: int) -> np.ndarray:
    g = np.arange(n, dtype=np.uint64)
    return (splitmix64(g ^ np.uint64((seed ^ 0x6D61736B) & 0xFFFFFFFFFFFFFFFF)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def plaintext(seed: int, g: int, length: int) -> bytes:
    """Host copy of the generator's payload plaintext for frame g (small sizes only)."""
    with np.errstate(over="ignore"):
        base = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ (np.uint64(g) * GOLDEN)
        words = splitmix64(base + np.arange((length + 7) // 8, dtype=np.uint64))
    return words.view(np.uint8)[:length].tobytes()


def header_len(length: np.ndarray, masked: np.ndarray, len_form: np.ndarray) -> np.ndarray:
    ext = np.where(len_form == 7, 0, np.where(len_form == 16, 2, 8))
    return 2 + ext + 4 * masked.astype(np.int64)


def min_len_form(length: np.ndarray) -> np.ndarray:
    return np.where(length <= 125, 7, np.where(length <= 0xFFFF, 16, 64)).astype(np.uint8)


@dataclass
class Layout:
    name: str
    desc: np.ndarray        # SYNTH_DTYPE [n_frames]
    conns: np.ndarray       # int64 [n_conns, 2] = (off, len)
    arena_bytes: int        # input bytes (without IN_PAD)
    payload_len: int        # sum of payload lengths
    payload_padded: int     # output arena bytes (16-byte rounded lengths)
    seed: int

    @property
    def n_frames(self) -> int:
        return int(self.desc.shape[0])

    @property
    def n_conns(self) -> int:
        return int(self.conns.shape[0])

    @property
    def header_bytes(self) -> int:
        return self.arena_bytes - self.payload_len

    def algorithmic_bytes(self) -> int:
        """SURVEY.md §8d per-frame figure h + 2L, summed: read h + L, write L."""
        return self.header_bytes + 2 * self.payload_len


def _assemble(name: str, lengths_per_conn, b0_per_conn, masked_per_conn, seed: int,
              len_form_per_conn=None) -> Layout:
    lengths = np.concatenate(lengths_per_conn).astype(np.uint64) if lengths_per_conn else np.zeros(0, np.uint64)
    b0 = np.concatenate(b0_per_conn).astype(np.uint8) if b0_per_conn else np.zeros(0, np.uint8)
    masked = np.concatenate(masked_per_conn).astype(np.uint8) if masked_per_conn else np.zeros(0, np.uint8)
    if len_form_per_conn is None:
        len_form = min_len_form(lengths)
    else:
        len_form = np.concatenate(len_form_per_conn).astype(np.uint8)
    h = header_len(lengths.astype(np.int64), masked, len_form.astype(np.int64))
    fsize = h.astype(np.uint64) + lengths
    counts = np.array([len(x) for x in lengths_per_conn], dtype=np.int64)
    starts = np.concatenate([[0], np.cumsum(fsize)]).astype(np.uint64)
    desc = np.zeros(lengths.shape[0], dtype=SYNTH_DTYPE)
    desc["hdr_off"] = starts[:-1]
    desc["length"] = lengths
    desc["mask"] = frame_masks(lengths.shape[0], seed)
    desc["b0"] = b0
    desc["len_form"] = len_form
    desc["masked"] = masked
    conn_first = np.concatenate([[0], np.cumsum(counts)])
    conns = np.zeros((counts.shape[0], 2), dtype=np.int64)
    conns[:, 0] = starts[conn_first[:-1]].astype(np.int64)
    conns[:, 1] = (starts[conn_first[1:]] - starts[conn_first[:-1]]).astype(np.int64)
    total = int(starts[-1])
    pl = int(lengths.sum())
    padded = int(((lengths + np.uint64(15)) // np.uint64(16) * np.uint64(16)).sum())
    return Layout(name, desc, conns, total, pl, padded, seed)


def uniform(n_conns: int, frames_per_conn: int, length: int, opcode: int = 0x2, masked: bool = True,
            seed: int = 0x67657600, name: str = "uniform") -> Layout:
    """C2 / C3: identical masked binary frames (FIN=1), vectorised layout."""
    n = n_conns * frames_per_conn
    lf = int(min_len_form(np.array([length]))[0])
    h = int(header_len(np.array([length]), np.array([int(masked)]), np.array([lf]))[0])
    fsize = h + length
    desc = np.zeros(n, dtype=SYNTH_DTYPE)
    desc["hdr_off"] = np.arange(n, dtype=np.uint64) * np.uint64(fsize)
    desc["length"] = length
    desc["mask"] = frame_masks(n, seed)
    desc["b0"] = 0x80 | opcode
    desc["len_form"] = lf
    desc["masked"] = int(masked)
    stream = frames_per_conn * fsize
    conns = np.zeros((n_conns, 2), dtype=np.int64)
    conns[:, 0] = np.arange(n_conns, dtype=np.int64) * stream
    conns[:, 1] = stream
    padded = n * ((length + 15) // 16 * 16)
    return Layout(name, desc, conns, n * fsize, n * length, padded, seed)


def config_c2(seed: int = 0x67657600, n_conns: int = 4096) -> Layout:
    """262 144 x 4 KiB masked binary frames (h = 8)."""
    return uniform(n_conns, 262144 // n_conns, 4096, seed=seed, name="C2: 262144 x 4 KiB masked binary")


def config_c3(seed: int = 0x67657600, n_conns: int = 16384, n_frames: int = 1 << 20) -> Layout:
    """1 048 576 x 64 KiB masked binary frames (h = 14): the HBM-roofline config."""
    return uniform(n_conns, n_frames // n_conns, 65536, seed=seed,
                   name=f"C3: {n_frames} x 64 KiB masked binary")


def config_c4(total_payload: int, n_conns: int = 8192, alpha: float = 1.1, lo: int = 64,
              hi: int = 1 << 20, seed: int = 0x67657604) -> Layout:
    """Bounded power-law (Pareto alpha) masked binary frames, many connections."""
    rng = np.random.default_rng(seed)
    per_conn = total_payload // n_conns
    lengths, b0s, ms = [], [], []
    for _ in range(n_conns):
        acc = []
        got = 0
        while got < per_conn:
            u = rng.random(4096)
            L = np.floor(lo * (1.0 - u * (1.0 - (lo / hi) ** alpha)) ** (-1.0 / alpha)).astype(np.int64)
            L = np.clip(L, lo, hi)
            cs = np.cumsum(L)
            k = int(np.searchsorted(cs, per_conn - got, side="left")) + 1
            L = L[:k]
            acc.append(L)
            got += int(L.sum())
        L = np.concatenate(acc)
        lengths.append(L)
        b0s.append(np.full(L.shape[0], 0x82, np.uint8))
        ms.append(np.ones(L.shape[0], np.uint8))
    return _assemble(f"C4: power-law {lo}B-{hi}B alpha={alpha}", lengths, b0s, ms, seed)


def config_c5(n_conns: int = 64, messages_per_conn: int = 4, message_bytes: int = 1 << 20,
              max_fragment: int = 65536, control_prob: float = 0.25, seed: int = 0x67657605) -> Layout:
    """1 MiB text messages as FIN=0 continuation chains with masked ping/pong
    control frames (0-125 B) interleaved between fragments."""
    rng = np.random.default_rng(seed)
    lengths, b0s, ms = [], [], []
    for _ in range(n_conns):
        L, B = [], []
        for _m in range(messages_per_conn):
            left = message_bytes
            first = True
            while left > 0:
                f = int(min(left, rng.integers(1, max_fragment + 1)))
                left -= f
                op = 0x1 if first else 0x0
                fin = 0x80 if left == 0 else 0x00
                L.append(f)
                B.append(fin | op)
                first = False
                if left > 0 and rng.random() < control_prob:
                    L.append(int(rng.integers(0, 126)))
                    B.append(0x80 | (0x9 if rng.random() < 0.5 else 0xA))
        lengths.append(np.array(L, np.int64))
        b0s.append(np.array(B, np.uint8))
        ms.append(np.ones(len(L), np.uint8))
    return _assemble("C5: fragmented text + ping/pong", lengths, b0s, ms, seed)


def shard_bounds(conn_lens: np.ndarray, world: int) -> list:
    """Connection index boundaries [b_0 = 0, ..., b_world = n]: rank r takes the
    connections whose cumulative stream bytes end in (r, r+1] * total / world."""
    n = int(conn_lens.shape[0])
    cum = np.cumsum(conn_lens)
    total = int(cum[-1]) if n else 0
    b = [0]
    for r in range(1, world):
        cut = -(-total * r // world)  # ceil
        b.append(max(b[-1], int(np.searchsorted(cum, cut, side="left")) + 1 if total else 0))
    b.append(n)
    return [min(x, n) for x in b]


def shard(layout: Layout, rank: int, world: int) -> Layout:
    """Connection -> GPU assignment: contiguous byte-balanced split of the
    connection list (greedy over the running byte count), so each rank decodes
    only its own connections' streams (gev's connection -> loop sharding,
    server.go:80-91, load_balance.go:7-28, lifted to connection -> GPU)."""
    if world == 1:
        return layout
    c0, c1 = shard_bounds(layout.conns[:, 1], world)[rank:rank + 2]
    if c1 <= c0:
        return Layout(layout.name, layout.desc[:0], layout.conns[:0], 0, 0, 0, layout.seed)
    off0 = int(layout.conns[c0, 0])
    off1 = int(layout.conns[c1 - 1, 0] + layout.conns[c1 - 1, 1])
    sel = (layout.desc["hdr_off"] >= off0) & (layout.desc["hdr_off"] < off1)
    desc = layout.desc[sel].copy()
    desc["hdr_off"] -= np.uint64(off0)
    conns = layout.conns[c0:c1].copy()
    conns[:, 0] -= off0
    pl = int(desc["length"].sum())
    padded = int(((desc["length"] + np.uint64(15)) // np.uint64(16) * np.uint64(16)).sum())
    return Layout(layout.name, desc, conns, off1 - off0, pl, padded, layout.seed)


def lpt_assign(conn_lens: np.ndarray, world: int) -> np.ndarray:
    """Greedy LPT (longest processing time first): connections in descending
    stream-byte order, each to the rank with the fewest bytes so far (ties to
    the lowest rank).  Returns the rank of every connection.  The largest
    rank's load is at most 4/3 of the optimum (Graham's bound)."""
    n = int(conn_lens.shape[0])
    owner = np.zeros(n, np.int64)
    if world <= 1 or n == 0:
        return owner
    import heapq
    heap = [(0, r) for r in range(world)]
    for c in np.argsort(-conn_lens.astype(np.int64), kind="stable"):
        load, r = heapq.heappop(heap)
        owner[c] = r
        heapq.heappush(heap, (load + int(conn_lens[c]), r))
    return owner


def shard_lpt(layout: Layout, rank: int, world: int) -> Layout:
    """Connection -> GPU assignment by greedy LPT over stream bytes (SURVEY.md
    §8d C4 / §8e): rank `rank` takes the connections lpt_assign gives it, in
    their original order, laid out back to back in its own arena.  Frame
    descriptors keep their global index order (synth payloads are keyed by the
    descriptor's position, so each rank's batch is self-consistent)."""
    if world == 1:
        return layout
    lens = layout.conns[:, 1]
    mine = np.nonzero(lpt_assign(lens, world) == rank)[0]
    if mine.size == 0:
        return Layout(layout.name, layout.desc[:0], layout.conns[:0], 0, 0, 0, layout.seed)
    hdr = layout.desc["hdr_off"].astype(np.int64)
    # frames of connection c are those with hdr_off in [off_c, off_c + len_c)
    first = np.searchsorted(hdr, layout.conns[mine, 0], side="left")
    last = np.searchsorted(hdr, layout.conns[mine, 0] + lens[mine], side="left")
    counts = last - first
    idx = np.concatenate([np.arange(a, b) for a, b in zip(first, last)]) if counts.sum() else np.zeros(0, np.int64)
    new_off = np.concatenate([[0], np.cumsum(lens[mine])])
    desc = layout.desc[idx].copy()
    shift = np.repeat(new_off[:-1] - layout.conns[mine, 0], counts)
    desc["hdr_off"] = (hdr[idx] + shift).astype(np.uint64)
    conns = np.stack([new_off[:-1], lens[mine]], axis=1).astype(np.int64)
    pl = int(desc["length"].sum())
    padded = int(((desc["length"] + np.uint64(15)) // np.uint64(16) * np.uint64(16)).sum())
    return Layout(layout.name, desc, conns, int(new_off[-1]), pl, padded, layout.seed)


def run_frames(layout: Layout) -> int:
    """summary.run_frames of a decode of the whole layout: frames whose size
    (h + L) equals the size of the frame before them on the same connection."""
    d = layout.desc
    if d.shape[0] == 0:
        return 0
    size = header_len(d["length"].astype(np.int64), d["masked"], d["len_form"].astype(np.int64)) + \
        d["length"].astype(np.int64)
    first = np.zeros(d.shape[0], bool)
    starts = np.searchsorted(d["hdr_off"].astype(np.int64), layout.conns[:, 0], side="left")
    first[starts[starts < d.shape[0]]] = True
    return int(((size[1:] == size[:-1]) & ~first[1:]).sum())


def size_histogram(layout: Layout) -> list:
    """Realised payload-length histogram, power-of-two buckets: [[lo, hi, frames], ...]."""
    L = layout.desc["length"].astype(np.int64)
    if L.size == 0:
        return []
    b = np.zeros(L.shape, np.int64)
    nz = L > 0
    b[nz] = np.floor(np.log2(L[nz])).astype(np.int64) + 1
    cnt = np.bincount(b)
    return [[0 if k == 0 else 1 << (k - 1), 0 if k == 0 else (1 << k) - 1, int(c)]
            for k, c in enumerate(cnt) if c]


def synth_host(layout: Layout) -> np.ndarray:
    """Host copy of the device generator's output (gevws_synth_async) for
    small layouts: used for the CPU baseline sample and to pin the device
    generator in tests.  Returns the arena (without IN_PAD)."""
    arena = np.zeros(layout.arena_bytes, np.uint8)
    d = layout.desc
    for g in range(d.shape[0]):
        off = int(d["hdr_off"][g])
        L = int(d["length"][g])
        lf = int(d["len_form"][g])
        masked = int(d["masked"][g])
        key = int(d["mask"][g])
        mb = 0x80 if masked else 0
        hdr = bytearray([int(d["b0"][g])])
        if lf == 7:
            hdr.append(mb | L)
        elif lf == 16:
            hdr += bytes([mb | 126]) + L.to_bytes(2, "big")
        else:
            hdr += bytes([mb | 127]) + L.to_bytes(8, "big")
        if masked:
            hdr += key.to_bytes(4, "little")
        h = len(hdr)
        arena[off:off + h] = np.frombuffer(bytes(hdr), np.uint8)
        p = np.frombuffer(plaintext(layout.seed, g, L), np.uint8)
        if masked:
            # key phase 0 at the payload start (ws.Cipher offset 0, protocol.go:54)
            q = np.zeros((L + 3) // 4 * 4, np.uint8)
            q[:L] = p
            q.view("<u4")[:] ^= np.uint32(key)
            p = q[:L]
        arena[off + h:off + h + L] = p
    return arena
