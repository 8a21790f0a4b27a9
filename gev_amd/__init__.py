"""gev_amd -- MI355X-native WebSocket frame-decode / payload-unmask engine.

Drop-in for the hot path of gev's websocket plugin
(plugins/websocket/protocol.go:27-64 ``Protocol.UnPacket``): the decode runs
in hand-written gfx950 HIP kernels (gev_amd/csrc/gevws_device.hip) behind the
C ABI of include/gevws.h.  This Python layer is a thin ctypes binding used by
the tests and bench; torch supplies device memory, streams and
torch.distributed (plumbing only).

Names mirror the reference: ``RingBuffer`` (github.com/Allenxuxu/ringbuffer as
gev uses it), ``Connection`` (gev.Connection's websocket context keys),
``Protocol.unpacket`` / ``Protocol.packet`` (websocket.Protocol),
``handler_protocol`` (Connection.handlerProtocol, connection.go:208-218).
"""
from __future__ import annotations

import ctypes
import atexit
import weakref
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import _abi
from ._abi import (ERR_CAPACITY, ERR_DEVICE, ERR_HANDSHAKE, ERR_INVALID, ERR_LEN_MSB, ERR_NOT_UPGRADED,
                   HANDSHAKE, IN_PAD, MEM_DEFAULT, MEM_FINE, MEM_UNCACHED, NEED_MORE, OK, PAYLOAD_ALIGN,
                   SUMMARY_UNORDERED, TILE, Header)

lib = _abi.load()

FRAME_DTYPE = np.dtype([("fin", "u1"), ("rsv", "u1"), ("opcode", "u1"), ("masked", "u1"),
                        ("mask", "u1", (4,)), ("length", "<i8"),
                        ("payload_off", "<u8"), ("src_off", "<u8")])
CONN_OUT_DTYPE = np.dtype([("first_frame", "<u8"), ("consumed", "<u8"), ("payload_base", "<u8"),
                           ("nframes", "<u4"), ("status", "<i4")])
SUMMARY_DTYPE = np.dtype([("frames", "<u8"), ("payload_bytes", "<u8"), ("payload_len", "<u8"),
                          ("errors", "<u8"), ("status", "<i4"), ("flags", "<u4"), ("run_frames", "<u8"),
                          ("reserved", "<u8", (2,))])
OUT_FRAME_DTYPE = np.dtype([("fin", "u1"), ("rsv", "u1"), ("opcode", "u1"), ("masked", "u1"),
                            ("mask", "u1", (4,)), ("length", "<i8"),
                            ("payload_off", "<u8"), ("payload_len", "<u8")])
SYNTH_DTYPE = np.dtype([("hdr_off", "<u8"), ("length", "<u8"), ("mask", "<u4"), ("b0", "u1"),
                        ("len_form", "u1"), ("masked", "u1"), ("pad", "u1")])
assert FRAME_DTYPE.itemsize == 32 and CONN_OUT_DTYPE.itemsize == 32
assert SUMMARY_DTYPE.itemsize == 64 and SYNTH_DTYPE.itemsize == 24


def status_string(st: int) -> str:
    return lib.gevws_status_string(st).decode()


def device_count() -> int:
    return lib.gevws_device_count()


def _torch():
    import torch
    return torch


def _stream_handle(stream) -> Optional[int]:
    if stream is None:
        return _torch().cuda.current_stream().cuda_stream
    return getattr(stream, "cuda_stream", stream)


@dataclass
class Batch:
    """Device-resident result of one batch decode (all tensors on the GPU)."""
    frames: "object"      # uint8 [max_frames, 32]  (gevws_frame records)
    payload: "object"     # uint8 [payload_cap + 16]
    conn_out: "object"    # uint8 [n_conns, 32]     (gevws_conn_out)
    summary: "object"     # uint8 [64]              (gevws_summary)
    n_conns: int
    aux_slots: int = 0    # close-reply slots reserved after the payload arena (alloc_batch)

    def summary_host(self) -> np.ndarray:
        return self.summary.cpu().numpy().view(SUMMARY_DTYPE)[0]

    def frames_host(self) -> np.ndarray:
        n = int(self.summary_host()["frames"])
        return self.frames[:n].cpu().numpy().reshape(-1).view(FRAME_DTYPE)

    def conn_out_host(self) -> np.ndarray:
        return self.conn_out[: self.n_conns].cpu().numpy().reshape(-1).view(CONN_OUT_DTYPE)

    def payload_host(self) -> np.ndarray:
        n = int(self.summary_host()["payload_bytes"])
        return self.payload[:n].cpu().numpy()


class _DevAddr:
    """A bare device address with the one method the launch wrappers read."""
    __slots__ = ("addr",)

    def __init__(self, addr: int):
        self.addr = addr

    def data_ptr(self) -> int:
        return self.addr


class PinnedArena:
    """Page-locked host memory mapped into the device (gevws_pinned_alloc):
    `host` is a numpy uint8 view for the CPU, `at(off)` a device address a
    decode can take as its payload arena, so the unmask kernel writes the
    plaintext straight into host memory (host-ingress helper, not on the
    reference path)."""

    def __init__(self, nbytes: int):
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        st = lib.gevws_pinned_alloc(nbytes, ctypes.byref(h), ctypes.byref(d))
        if st != OK:
            raise RuntimeError(f"gevws_pinned_alloc({nbytes}): {status_string(st)}")
        self.nbytes = nbytes
        self._h, self._d = h.value, d.value
        self.host = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self._h))

    def at(self, offset: int = 0) -> _DevAddr:
        if not 0 <= offset <= self.nbytes:
            raise ValueError(f"PinnedArena.at({offset}): outside {self.nbytes} bytes")
        return _DevAddr(self._d + offset)

    def data_ptr(self) -> int:
        return self._d

    def close(self) -> None:
        if self._h:
            self.host = None
            lib.gevws_pinned_free(self._h)
            self._h = self._d = None

    def __del__(self, _free=lib.gevws_pinned_free):  # bound now: module globals are gone at exit
        if getattr(self, "_h", None):
            _free(self._h)


# Objects still alive at interpreter exit (e.g. held by a failed test's
# traceback) are freed in dependency order -- protocols, then engines -- from
# an atexit hook, while the HIP runtime is still up; the garbage collector's
# order at shutdown is arbitrary, and a protocol freed after its engine would
# synchronise a destroyed stream.
_LIVE_PROTOCOLS: "weakref.WeakSet" = weakref.WeakSet()
_LIVE_ENGINES: "weakref.WeakSet" = weakref.WeakSet()


def _close_live() -> None:
    for p in list(_LIVE_PROTOCOLS):
        p.close()
    for e in list(_LIVE_ENGINES):
        e.close()


atexit.register(_close_live)


class Engine:
    """One gevws_ctx (one per event loop / rank) on one GPU."""

    def __init__(self, device: int = 0):
        if device_count() <= device:
            raise RuntimeError(f"gev_amd.Engine: no HIP device {device} (found {device_count()}); "
                               "the decode path has no CPU fallback")
        self.device = device
        self._ctx = lib.gevws_ctx_create(device)
        if not self._ctx:
            raise RuntimeError("gevws_ctx_create failed")
        _LIVE_ENGINES.add(self)

    def close(self):
        if self._ctx:
            lib.gevws_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------- tuning
    def set_tuning(self, key: int, value: int) -> None:
        st = lib.gevws_ctx_set_tuning(self._ctx, key, value)
        if st != OK:
            raise ValueError(f"set_tuning({key}, {value}): {status_string(st)}")

    # -------------------------------------------------------------- stream ordering
    def order_after_last(self, stream=None) -> None:
        """Make `stream` (default: torch's current stream) wait for this
        context's last call, whichever stream it ran on."""
        st = lib.gevws_ctx_order_after_last(self._ctx, _stream_handle(stream))
        if st != OK:
            raise RuntimeError(f"gevws_ctx_order_after_last: {status_string(st)}")

    @property
    def last_unmask_grid(self) -> int:
        """Workgroups of the last multi-kernel decode's unmask launch."""
        return int(lib.gevws_ctx_last_unmask_grid(self._ctx))

    @property
    def last_split_lanes(self) -> int:
        """Lanes per connection of the last multi-kernel decode's header walk (1 = not split)."""
        return int(lib.gevws_ctx_last_split_lanes(self._ctx))

    @property
    def last_split_fallbacks(self) -> int:
        """Connections the last multi-kernel decode's split walk re-walked
        serially after a missed guess (0 when not split; waits for the decode)."""
        return int(lib.gevws_ctx_last_split_fallbacks(self._ctx))

    @staticmethod
    def variant_name(i: int, key: int = _abi.TUNE_UNMASK_VARIANT) -> Optional[str]:
        n = lib.gevws_tuning_name(key, i)
        return n.decode() if n else None

    @staticmethod
    def variants(key: int = _abi.TUNE_UNMASK_VARIANT) -> List[int]:
        """Every valid value of a variant knob (GEVWS_TUNE_UNMASK_VARIANT / _WALK_VARIANT)."""
        out = []
        while Engine.variant_name(len(out), key) is not None:
            out.append(len(out))
        return out

    # -------------------------------------------------------------- timing
    def set_timing(self, enable: bool):
        lib.gevws_ctx_set_timing(self._ctx, int(enable))

    def timing(self) -> Tuple[Tuple[float, float, float, float], int]:
        """(summed ms per phase [walk-count, scan, walk-emit, unmask], calls) since the last query."""
        ms = (ctypes.c_float * 4)()
        calls = ctypes.c_uint32()
        st = lib.gevws_ctx_timing(self._ctx, ms, ctypes.byref(calls))
        if st != OK:
            raise RuntimeError(status_string(st))
        return tuple(ms), calls.value

    # -------------------------------------------------------------- decode
    def alloc_batch(self, n_conns: int, max_frames: int, payload_cap: int, aux_slots: int = 0) -> Batch:
        """Output buffers; aux_slots reserves room after the payload arena for
        close-reply bodies (Engine.serve)."""
        torch = _torch()
        dev = torch.device("cuda", self.device)
        extra = (aux_slots * _abi.AUX_SLOT + 128) if aux_slots else 0
        return Batch(frames=torch.empty((max(max_frames, 1), 32), dtype=torch.uint8, device=dev),
                     payload=torch.empty(payload_cap + 16 + extra, dtype=torch.uint8, device=dev),
                     conn_out=torch.empty((max(n_conns, 1), 32), dtype=torch.uint8, device=dev),
                     summary=torch.zeros(64, dtype=torch.uint8, device=dev), n_conns=n_conns, aux_slots=aux_slots)

    def decode_async(self, arena, in_bytes: int, conns, n_conns: int, out: Batch, max_frames: int,
                     payload_cap: int, stream=None) -> None:
        """gevws_decode_batch_async on device tensors (arena: uint8 with IN_PAD slack;
        conns: int64 [n,2] = (off, len))."""
        st = lib.gevws_decode_batch_async(
            self._ctx, _stream_handle(stream), arena.data_ptr(), in_bytes,
            conns.data_ptr() if n_conns else None, n_conns, out.frames.data_ptr(), max_frames,
            out.payload.data_ptr(), payload_cap, out.conn_out.data_ptr(), out.summary.data_ptr())
        if st != OK:
            raise RuntimeError(f"gevws_decode_batch_async: {status_string(st)}")

    def decode_post(self, arena, in_bytes: int, conns, n_conns: int, out: Batch, max_frames: int,
                    payload_cap: int) -> None:
        """gevws_decode_batch_post: a live pass on the context's stream, posted
        to the resident decode service when it is on (set_service) and the
        pass fits it, else launched; completion_seq tells which word to wait for."""
        st = lib.gevws_decode_batch_post(
            self._ctx, arena.data_ptr(), in_bytes, conns.data_ptr() if n_conns else None, n_conns,
            out.frames.data_ptr(), max_frames, out.payload.data_ptr(), payload_cap, out.conn_out.data_ptr(),
            out.summary.data_ptr())
        if st != OK:
            raise RuntimeError(f"gevws_decode_batch_post: {status_string(st)}")

    def set_service(self, on: bool) -> None:
        """gevws_ctx_set_service: the resident decode service (False stops it)."""
        st = lib.gevws_ctx_set_service(self._ctx, 1 if on else 0)
        if st != OK:
            raise RuntimeError(f"gevws_ctx_set_service: {status_string(st)}")

    def service_stop(self) -> None:
        """gevws_ctx_service_stop: end the live instance (the next post starts another)."""
        lib.gevws_ctx_service_stop(self._ctx)

    def set_direct(self, on: bool) -> None:
        """gevws_ctx_set_direct: live passes written into the context's own AQL queue."""
        st = lib.gevws_ctx_set_direct(self._ctx, 1 if on else 0)
        if st != OK:
            raise RuntimeError(f"gevws_ctx_set_direct: {status_string(st)}")

    @property
    def direct_dispatches(self) -> int:
        """gevws_ctx_direct_dispatches: passes written into the context's own queue so far."""
        return int(lib.gevws_ctx_direct_dispatches(self._ctx))

    def synchronize(self) -> None:
        """gevws_ctx_synchronize: everything the context enqueued (stream, own queue, service)."""
        st = lib.gevws_ctx_synchronize(self._ctx)
        if st != OK:
            raise RuntimeError(f"gevws_ctx_synchronize: {status_string(st)}")

    def service_stats(self) -> dict:
        """gevws_ctx_service_stats: service instances launched, passes posted to them."""
        la, po = ctypes.c_int64(), ctypes.c_int64()
        lib.gevws_ctx_service_stats(self._ctx, ctypes.byref(la), ctypes.byref(po))
        return {"launches": la.value, "posts": po.value}

    def decode(self, arena, in_bytes: int, conns, n_conns: int, max_frames: Optional[int] = None,
               payload_cap: Optional[int] = None, stream=None, aux_slots: int = 0) -> Batch:
        """Decode a device-resident batch; grows capacities once on ERR_CAPACITY.
        aux_slots reserves close-reply space for a following Engine.serve."""
        torch = _torch()
        if max_frames is None:
            max_frames = min(in_bytes // 2 + 1, 0xFFFFFFFF)
        if payload_cap is None:
            payload_cap = in_bytes + 16 * min(max_frames, in_bytes // 64 + 64) + 64
        for attempt in range(2):
            out = self.alloc_batch(n_conns, max_frames, payload_cap, aux_slots)
            self.decode_async(arena, in_bytes, conns, n_conns, out, max_frames, payload_cap, stream)
            torch.cuda.synchronize(self.device)
            s = out.summary_host()
            if int(s["status"]) == ERR_CAPACITY and attempt == 0:
                max_frames = max(int(s["frames"]), 1)
                payload_cap = max(int(s["payload_bytes"]), 16)
                continue
            if int(s["status"]) != OK:
                raise RuntimeError(f"decode: {status_string(int(s['status']))}")
            return out
        raise RuntimeError("decode: capacity retry failed")

    def encode_async(self, frames_dev, n: int, payload, out, out_cap: int, out_off, summary, stream=None) -> None:
        """gevws_encode_batch_async: FrameToBytes for n records (OUT_FRAME_DTYPE rows as a
        uint8 [n, 32] device tensor) into `out` (>= out_cap + OUT_PAD bytes)."""
        st = lib.gevws_encode_batch_async(self._ctx, _stream_handle(stream), frames_dev.data_ptr() if n else None,
                                          n, payload.data_ptr(), out.data_ptr(), out_cap,
                                          out_off.data_ptr(), summary.data_ptr())
        if st != OK:
            raise RuntimeError(f"gevws_encode_batch_async: {status_string(st)}")

    def encode(self, frames: np.ndarray, payload, out_cap: Optional[int] = None):
        """Encode host records (OUT_FRAME_DTYPE) whose payloads live in the device
        tensor `payload`; returns (wire device tensor [total], out_off numpy)."""
        torch = _torch()
        dev = torch.device("cuda", self.device)
        n = int(frames.shape[0])
        if out_cap is None:
            out_cap = int(frames["payload_len"].sum()) + 14 * n
        fr = torch.from_numpy(np.ascontiguousarray(frames).view(np.uint8).reshape(-1, 32).copy()).to(dev) \
            if n else torch.zeros((1, 32), dtype=torch.uint8, device=dev)
        out = torch.empty(out_cap + _abi.OUT_PAD, dtype=torch.uint8, device=dev)
        off = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        summ = torch.zeros(64, dtype=torch.uint8, device=dev)
        self.encode_async(fr, n, payload, out, out_cap, off, summ)
        torch.cuda.synchronize(self.device)
        s = summ.cpu().numpy().view(SUMMARY_DTYPE)[0]
        if int(s["status"]) != OK:
            raise RuntimeError(f"encode: {status_string(int(s['status']))}")
        return out[: int(s["payload_bytes"])], off[:n].cpu().numpy().astype(np.uint64)

    def dispatch_async(self, frames_dev, n: int, policy: int, payload, aux_off: int, aux_cap: int, replies,
                       reply_of, summary, stream=None) -> None:
        """gevws_dispatch_async: HandlerWrap.OnMessage replies for n decoded frames."""
        st = lib.gevws_dispatch_async(self._ctx, _stream_handle(stream), frames_dev.data_ptr() if n else None, n,
                                      policy, payload.data_ptr(), aux_off, aux_cap,
                                      replies.data_ptr(), reply_of.data_ptr(), summary.data_ptr())
        if st != OK:
            raise RuntimeError(f"gevws_dispatch_async: {status_string(st)}")

    def serve(self, out: "Batch", policy: int, aux_slots: Optional[int] = None):
        """One server step after a decode: dispatch (wrap.go:38-90) + encode of
        the replies.  `out.payload` must have room for the close-reply bodies
        after the decoded payloads (see alloc_batch(aux_slots=...)).  Returns
        (wire device tensor, reply_of numpy, summary of the dispatch)."""
        torch = _torch()
        dev = torch.device("cuda", self.device)
        s = out.summary_host()
        n = int(s["frames"])
        aux_off = (int(s["payload_bytes"]) + 127) // 128 * 128
        aux_cap = out.payload.numel() - 16 - aux_off
        replies = torch.empty((max(n, 1), 32), dtype=torch.uint8, device=dev)
        reply_of = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        dsum = torch.zeros(64, dtype=torch.uint8, device=dev)
        self.dispatch_async(out.frames, n, policy, out.payload, aux_off, max(aux_cap, 0), replies, reply_of, dsum)
        torch.cuda.synchronize(self.device)
        ds = dsum.cpu().numpy().view(SUMMARY_DTYPE)[0]
        if int(ds["status"]) != OK:
            raise RuntimeError(f"dispatch: {status_string(int(ds['status']))}")
        nr = int(ds["frames"])
        rep_host = replies[:nr].cpu().numpy().reshape(-1).view(OUT_FRAME_DTYPE)
        wire, _ = self.encode(rep_host, out.payload, int(rep_host["payload_len"].sum()) + 14 * nr)
        return wire, reply_of[:n].cpu().numpy(), ds

    def set_completion_flag(self, arena: Optional["PinnedArena"], offset: int = 0) -> None:
        """gevws_ctx_set_completion_flag: the one-launch kernels store their
        sequence number into the 32-bit word at arena.host[offset:offset+4]
        (None: off)."""
        addr = arena.at(offset).data_ptr() if arena is not None else None
        st = lib.gevws_ctx_set_completion_flag(self._ctx, addr)
        if st != OK:
            raise RuntimeError(f"gevws_ctx_set_completion_flag: {status_string(st)}")

    def set_timeline_ticks(self, arena: Optional["PinnedArena"], offset: int = 0) -> None:
        """gevws_ctx_set_timeline_ticks: the one-launch kernels stamp their start /
        end ticks (GPU constant-rate clock) into 4 u64 at arena.host[offset:offset+32]
        before they signal (None: off)."""
        addr = arena.at(offset).data_ptr() if arena is not None else None
        st = lib.gevws_ctx_set_timeline_ticks(self._ctx, addr)
        if st != OK:
            raise RuntimeError(f"gevws_ctx_set_timeline_ticks: {status_string(st)}")

    @property
    def completion_seq(self) -> int:
        """gevws_ctx_completion_seq: the number the last call's last kernel
        stores into the completion word, -1 when it does not signal."""
        return int(lib.gevws_ctx_completion_seq(self._ctx))

    def handle_decoded(self, out: "Batch", policy: int, max_frames: int, aux_slots: int, out_cap: int):
        """gevws_handle_decoded_async: dispatch + encode of the replies chained
        behind the decode with no host round trip (one launch when max_frames
        <= 1 024).  Returns (wire device tensor, reply_of numpy, dispatch
        summary, encode summary)."""
        torch = _torch()
        dev = torch.device("cuda", self.device)
        # the close bodies go into the slots alloc_batch reserved behind the
        # payload arena, never over decoded payloads the replies still read
        if not 0 <= aux_slots <= out.aux_slots:
            raise ValueError(f"handle_decoded: aux_slots {aux_slots} outside the batch's {out.aux_slots} reserved slots")
        aux_off = (out.payload.numel() - 16 - 128 * aux_slots) // 16 * 16
        n = max(int(max_frames), 1)
        replies = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        reply_of = torch.full((n,), -7, dtype=torch.int64, device=dev)
        sums = torch.zeros(128, dtype=torch.uint8, device=dev)
        wire = torch.zeros(out_cap + _abi.OUT_PAD, dtype=torch.uint8, device=dev)
        off = torch.empty(n, dtype=torch.int64, device=dev)
        st = lib.gevws_handle_decoded_async(self._ctx, None, out.frames.data_ptr(), int(max_frames),
                                            out.summary.data_ptr(), int(policy), out.payload.data_ptr(), aux_off,
                                            128 * aux_slots, replies.data_ptr(), reply_of.data_ptr(),
                                            sums.data_ptr(), wire.data_ptr(), int(out_cap), off.data_ptr(),
                                            sums.data_ptr() + 64)
        if st != OK:
            raise RuntimeError(f"gevws_handle_decoded_async: {status_string(st)}")
        torch.cuda.synchronize(self.device)
        ss = sums.cpu().numpy().view(SUMMARY_DTYPE)
        nf = int(out.summary_host()["frames"])
        return wire[: int(ss[1]["payload_bytes"])], reply_of[:nf].cpu().numpy(), ss[0], ss[1]

    def cipher_(self, buf, mask: bytes, offset: int = 0, nbytes: Optional[int] = None,
                byte_offset: int = 0, stream=None) -> None:
        """ws.Cipher (cipher.go:14-53) in place on a device uint8 tensor region."""
        m = (ctypes.c_uint8 * 4)(*mask)
        n = buf.numel() - byte_offset if nbytes is None else nbytes
        st = lib.gevws_cipher_async(self._ctx, _stream_handle(stream), buf.data_ptr() + byte_offset, n, m,
                                    offset)
        if st != OK:
            raise RuntimeError(status_string(st))

    def copy_(self, dst, src, nbytes: int, dst_offset: int = 0, src_offset: int = 0, grid: int = 0,
              stream=None) -> None:
        """gevws_copy_async: the streaming-copy ceiling kernel (measurement only)."""
        assert dst_offset + nbytes <= dst.numel() and src_offset + nbytes <= src.numel()
        st = lib.gevws_copy_async(self._ctx, _stream_handle(stream), dst.data_ptr() + dst_offset,
                                  src.data_ptr() + src_offset, nbytes, grid)
        if st != OK:
            raise RuntimeError(status_string(st))

    def synth(self, arena, desc_dev, n_frames: int, seed: int, stream=None) -> None:
        st = lib.gevws_synth_async(self._ctx, _stream_handle(stream), arena.data_ptr(), desc_dev.data_ptr(),
                                   n_frames, seed)
        if st != OK:
            raise RuntimeError(status_string(st))

    def verify(self, desc_dev, n_frames: int, seed: int, out: Batch, mismatch_dev, stream=None) -> None:
        if out.frames.shape[0] < n_frames:
            raise ValueError("verify: batch holds fewer frame records than the layout")
        st = lib.gevws_synth_verify_async(self._ctx, _stream_handle(stream), desc_dev.data_ptr(), n_frames,
                                          seed, out.frames.data_ptr(), out.payload.data_ptr(),
                                          out.payload.numel() - 16, mismatch_dev.data_ptr())
        if st != OK:
            raise RuntimeError(status_string(st))


# ====================================================================== host mirror
class RingBuffer:
    """ringbuffer.RingBuffer as gev uses it (New / Write / Length / PeekAll / Retrieve)."""

    def __init__(self, size: int = 4096):
        self._p = lib.gevws_ring_new(size)

    def __del__(self, _free=lib.gevws_ring_free):  # bound now: module globals are gone at exit
        if getattr(self, "_p", None):
            _free(self._p)
            self._p = None

    def write(self, data: bytes) -> int:
        buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data) if data else None
        return lib.gevws_ring_write(self._p, buf, len(data))

    def length(self) -> int:
        return lib.gevws_ring_length(self._p)

    def capacity(self) -> int:
        return lib.gevws_ring_capacity(self._p)

    def is_empty(self) -> bool:
        return self.length() == 0

    def peek_all(self) -> Tuple[bytes, bytes]:
        a, b = _abi.U8P(), _abi.U8P()
        na, nb = ctypes.c_uint64(), ctypes.c_uint64()
        lib.gevws_ring_peek_all(self._p, ctypes.byref(a), ctypes.byref(na), ctypes.byref(b), ctypes.byref(nb))
        first = ctypes.string_at(a, na.value) if na.value else b""
        end = ctypes.string_at(b, nb.value) if nb.value else b""
        return first, end

    def retrieve(self, n: int) -> None:
        lib.gevws_ring_retrieve(self._p, n)


_CONNS: "weakref.WeakValueDictionary[int, Connection]" = weakref.WeakValueDictionary()


class Connection:
    """The per-connection context keys of the websocket plugin (protocol.go:11-14)."""

    def __init__(self, upgraded: bool = True):
        self._p = lib.gevws_conn_new()
        _CONNS[self._p] = self
        self.set_upgraded(upgraded)

    def __del__(self, _free=lib.gevws_conn_free):  # bound now: module globals are gone at exit
        if getattr(self, "_p", None):
            _free(self._p)
            self._p = None

    def handshake(self) -> "HandshakeInfo":
        """The last handshake's ws.Handshake and error (after UnPacket ran it)."""
        hs = _abi.Handshake()
        lib.gevws_conn_handshake(self._p, ctypes.byref(hs))
        return HandshakeInfo._from(hs)

    def set_upgraded(self, v: bool) -> None:
        lib.gevws_conn_set_upgraded(self._p, int(v))

    @property
    def upgraded(self) -> bool:
        return bool(lib.gevws_conn_upgraded(self._p))

    def pending(self) -> int:
        return lib.gevws_conn_pending(self._p)


class RejectError(Exception):
    """ws.RejectConnectionError(RejectionStatus(code), RejectionReason(reason),
    RejectionHeader(header)) (plugins/websocket/ws/errors.go:81-129).  Raise it
    from an Upgrader hook; any other exception is a plain Go error (HTTP 500,
    ws.go:325-333)."""

    def __init__(self, reason: str = "", code: int = 0, header: bytes = b""):
        super().__init__(reason)
        self.reason, self.code, self.header = reason, code, header


class HandshakeError(Exception):
    """A failed Upgrader.Upgrade: kind = GEVWS_HS_*, reason = err.Error()."""

    def __init__(self, kind: int, reason: str, http_code: int):
        super().__init__(reason)
        self.kind, self.reason, self.http_code = kind, reason, http_code


@dataclass
class HandshakeInfo:
    """ws.Handshake (ws/ws.go:40-47) plus the error of the call."""
    protocol: bytes
    extensions: bytes
    error: int
    http_code: int
    reason: str

    @staticmethod
    def _from(hs: "_abi.Handshake") -> "HandshakeInfo":
        return HandshakeInfo(ctypes.string_at(hs.protocol, hs.protocol_len) if hs.protocol_len else b"",
                             ctypes.string_at(hs.extensions, hs.extensions_len) if hs.extensions_len else b"",
                             hs.error, hs.http_code, (hs.reason or b"").decode())


def accept_key(nonce: bytes) -> bytes:
    """initAcceptFromNonce (ws/nonce.go:23-39) through the C ABI."""
    assert len(nonce) == 24
    out = ctypes.create_string_buffer(28)
    lib.gevws_accept_key(nonce, out)
    return out.raw


class Upgrader:
    """ws.Upgrader (plugins/websocket/ws/ws.go:49-154) over the C ABI.

    Hooks take the reference's arguments (bytes for []byte):
      protocol(token) -> bool;  protocol_custom(conn, value) -> (selected, ok);
      extension(name, [(key, value or None)]) -> bool;
      extension_custom(conn, value, selected_so_far) -> (selected, ok);
      on_request(conn, uri), on_host(conn, host), on_header(conn, key, value):
        return None to accept, raise RejectError / Exception to reject;
      on_before_upgrade(conn) -> extra response header bytes or None, or raise.
    ``header`` is Upgrader.Header (raw "Key: value\\r\\n" lines)."""

    def __init__(self, header: bytes = b"", **hooks):
        self._p = lib.gevws_upgrader_new()
        self._keep: list = []
        if header:
            lib.gevws_upgrader_set_header(self._p, header, len(header))
        unknown = set(hooks) - {"protocol", "protocol_custom", "extension", "extension_custom", "on_request",
                                "on_host", "on_header", "on_before_upgrade"}
        if unknown:
            raise TypeError(f"unknown Upgrader hooks {sorted(unknown)}")
        self._hooks = hooks
        h = _abi.UpgraderHooks()
        for name, fn in hooks.items():
            if fn is not None:
                setattr(h, name, getattr(self, "_c_" + name)())
        self._cstruct = h
        lib.gevws_upgrader_set_hooks(self._p, ctypes.byref(h))

    def __del__(self, _free=lib.gevws_upgrader_free):  # bound now: module globals are gone at exit
        if getattr(self, "_p", None):
            _free(self._p)
            self._p = None

    # -- C trampolines (each keeps its own ctypes callback object alive)
    def _hold(self, b: bytes) -> int:
        buf = ctypes.create_string_buffer(b, len(b) + 1)
        self._keep.append(buf)
        return ctypes.addressof(buf)

    def _reject(self, rej, e: Exception) -> int:
        r = rej.contents
        if isinstance(e, RejectError):
            reason = e.reason.encode()
            r.code, r.plain = e.code, 0
            if e.header:
                r.header, r.header_len = self._hold(e.header), len(e.header)
        else:
            reason = str(e).encode()
            r.code, r.plain = 0, 1
        r.reason, r.reason_len = self._hold(reason), len(reason)
        return 1

    @staticmethod
    def _b(p, n) -> bytes:
        return ctypes.string_at(p, n) if n else b""

    def _c_protocol(self):
        fn = self._hooks["protocol"]
        return _abi.HOOK_PROTOCOL(lambda u, t, n: int(bool(fn(self._b(t, n)))))

    def _c_protocol_custom(self):
        fn = self._hooks["protocol_custom"]

        def cb(u, c, v, n, sel, sel_n):
            got, ok = fn(_CONNS.get(c), self._b(v, n))
            got = got.encode() if isinstance(got, str) else (got or b"")
            sel[0], sel_n[0] = (self._hold(got) if got else None), len(got)
            return int(bool(ok))
        return _abi.HOOK_PROTOCOL_CUSTOM(cb)

    def _c_extension(self):
        fn = self._hooks["extension"]

        def cb(u, name, n, params, npar):
            ps = [(self._b(params[i].key, params[i].key_len),
                   None if not params[i].value else self._b(params[i].value, params[i].value_len))
                  for i in range(npar)]
            return int(bool(fn(self._b(name, n), ps)))
        return _abi.HOOK_EXTENSION(cb)

    def _c_extension_custom(self):
        fn = self._hooks["extension_custom"]

        def cb(u, c, v, n, cur, cur_n, sel, sel_n):
            got, ok = fn(_CONNS.get(c), self._b(v, n), self._b(cur, cur_n))
            got = got or b""
            sel[0], sel_n[0] = (self._hold(got) if got else None), len(got)
            return int(bool(ok))
        return _abi.HOOK_EXTENSION_CUSTOM(cb)

    def _value_hook(self, name):
        fn = self._hooks[name]

        def cb(u, c, v, n, rej):
            try:
                fn(_CONNS.get(c), self._b(v, n))
                return 0
            except Exception as e:  # noqa: BLE001 -- every hook error is a rejection
                return self._reject(rej, e)
        return _abi.HOOK_ON_VALUE(cb)

    def _c_on_request(self):
        return self._value_hook("on_request")

    def _c_on_host(self):
        return self._value_hook("on_host")

    def _c_on_header(self):
        fn = self._hooks["on_header"]

        def cb(u, c, k, kn, v, vn, rej):
            try:
                fn(_CONNS.get(c), self._b(k, kn), self._b(v, vn))
                return 0
            except Exception as e:  # noqa: BLE001
                return self._reject(rej, e)
        return _abi.HOOK_ON_HEADER(cb)

    def _c_on_before_upgrade(self):
        fn = self._hooks["on_before_upgrade"]

        def cb(u, c, hdr, hdr_len, rej):
            try:
                extra = fn(_CONNS.get(c))
                if extra:
                    hdr[0], hdr_len[0] = self._hold(extra), len(extra)
                return 0
            except Exception as e:  # noqa: BLE001
                return self._reject(rej, e)
        return _abi.HOOK_ON_BEFORE_UPGRADE(cb)

    def upgrade(self, c: "Connection", buffer: "RingBuffer") -> Tuple[bytes, HandshakeInfo, Optional[HandshakeError]]:
        """Upgrade(c, in) -> (out, hs, err) (ws.go:158-343)."""
        self._keep.clear()
        out = _abi.U8P()
        n = ctypes.c_uint64()
        hs = _abi.Handshake()
        st = lib.gevws_upgrader_upgrade(self._p, c._p, buffer._p, ctypes.byref(out), ctypes.byref(n),
                                        ctypes.byref(hs))
        if st not in (OK, ERR_HANDSHAKE):
            raise RuntimeError(f"upgrade: {status_string(st)}")
        info = HandshakeInfo._from(hs)
        data = ctypes.string_at(out, n.value) if n.value else b""
        err = None if st == OK else HandshakeError(info.error, info.reason, info.http_code)
        return data, info, err


class DeviceArena:
    """gevws_device_alloc: zeroed device memory of a chosen kind (default,
    fine-grained or uncached); `data_ptr()` / `at(off)` for the launch
    wrappers (measurement helper: where the input arena lives)."""

    def __init__(self, device: int, nbytes: int, kind: int = 0):
        p = ctypes.c_void_p()
        st = lib.gevws_device_alloc(device, nbytes, kind, ctypes.byref(p))
        if st != OK:
            raise RuntimeError(f"gevws_device_alloc({nbytes}, kind {kind}): {status_string(st)}")
        self.device, self.nbytes, self.kind, self._p = device, nbytes, kind, p.value

    def data_ptr(self) -> int:
        return self._p

    def at(self, offset: int = 0) -> _DevAddr:
        if not 0 <= offset <= self.nbytes:
            raise ValueError(f"DeviceArena.at({offset}): outside {self.nbytes} bytes")
        return _DevAddr(self._p + offset)

    def close(self) -> None:
        if getattr(self, "_p", None):
            lib.gevws_device_free(self.device, self._p)
            self._p = None

    def __del__(self, _free=lib.gevws_device_free):
        if getattr(self, "_p", None):
            _free(self.device, self._p)


class Comm:
    """gevws_comm: an RCCL communicator over several GPUs of ONE process (a gev
    server whose event loops are placed on the node's devices round-robin) and
    the decode path's one collective, the all-reduce(sum) of every device's
    decoded {frames, payload bytes, errors}."""

    def __init__(self, devices: Sequence[int]):
        arr = (ctypes.c_int * len(devices))(*devices)
        self._p = lib.gevws_comm_create(arr, len(devices))
        if not self._p:
            raise RuntimeError(f"gevws_comm_create({list(devices)}) failed (RCCL missing or device not visible)")
        self.devices = list(devices)

    def __del__(self, _free=lib.gevws_comm_destroy):
        if getattr(self, "_p", None):
            _free(self._p)
            self._p = None

    def size(self) -> int:
        return int(lib.gevws_comm_size(self._p))

    def allreduce_counts(self, engines: Sequence["Engine"], batches: Sequence["Batch"]) -> Tuple[int, int, int]:
        """gevws_counts_allreduce over each device's last decode summary; every
        device's batch gets the totals in `counts` (int64[3] on its device);
        returns (frames, payload_len, errors) summed over the devices."""
        import torch
        n = len(self.devices)
        if len(engines) != n or len(batches) != n:
            raise ValueError("one engine and one batch per device of the communicator")
        # written only by the contexts' streams (no fill on torch's stream); the
        # blocks may have been freed by work still queued on torch's current
        # stream, so that stream is drained first (this is the synchronous form)
        counts = [torch.empty(3, dtype=torch.int64, device=torch.device("cuda", e.device)) for e in engines]
        for e in engines:
            torch.cuda.current_stream(torch.device("cuda", e.device)).synchronize()
        ctxs = (ctypes.c_void_p * n)(*[e._ctx for e in engines])
        sums = (ctypes.c_void_p * n)(*[b.summary.data_ptr() for b in batches])
        cnts = (ctypes.c_void_p * n)(*[c.data_ptr() for c in counts])
        tot = (ctypes.c_int64 * 3)()
        st = lib.gevws_counts_allreduce(self._p, ctxs, sums, cnts, tot)
        if st != OK:
            raise RuntimeError(f"gevws_counts_allreduce: {status_string(st)}")
        for b, c in zip(batches, counts):
            b.counts = c
        return int(tot[0]), int(tot[1]), int(tot[2])


class Protocol:
    """websocket.Protocol (plugins/websocket/protocol.go:16-69) over the device engine."""

    def __init__(self, engine: Engine, upgrader: Optional[Upgrader] = None):
        self.engine = engine
        self._p = lib.gevws_protocol_new(engine._ctx)
        _LIVE_PROTOCOLS.add(self)
        self.upgrader = upgrader
        if upgrader is not None:
            lib.gevws_protocol_set_upgrader(self._p, upgrader._p)

    def __del__(self, _free=lib.gevws_protocol_free):  # bound now: module globals are gone at exit
        if getattr(self, "_p", None):
            _free(self._p)
            self._p = None

    def close(self) -> None:
        """Free the protocol (it synchronises its engine's stream, so it must go
        before the engine: _close_live does protocols first at exit)."""
        if getattr(self, "_p", None):
            lib.gevws_protocol_free(self._p)
            self._p = None

    def unpacket(self, c: Connection, buffer: RingBuffer) -> Tuple[Optional[Header], Optional[bytes]]:
        """UnPacket(c, buffer) -> (ctx, out): one frame; (None, response) for
        the handshake (protocol.go:29-37); or (None, None)."""
        if self.upgrader is not None:
            self.upgrader._keep.clear()
        h = Header()
        out = _abi.U8P()
        n = ctypes.c_uint64()
        st = lib.gevws_protocol_unpacket(self._p, c._p, buffer._p, ctypes.byref(h), ctypes.byref(out),
                                         ctypes.byref(n))
        self.last_status = st
        if st in (HANDSHAKE, ERR_HANDSHAKE):
            return None, (ctypes.string_at(out, n.value) if n.value else None)
        if st != OK:
            return None, None
        return h, (ctypes.string_at(out, n.value) if n.value else b"")

    def unpacket_batch(self, conns: Sequence[Connection], buffers: Sequence[RingBuffer]) -> int:
        n = len(conns)
        cs = (ctypes.c_void_p * n)(*[c._p for c in conns])
        rs = (ctypes.c_void_p * n)(*[b._p for b in buffers])
        r = lib.gevws_protocol_unpacket_batch(self._p, cs, rs, n)
        if r < 0:
            raise RuntimeError(f"unpacket_batch: {status_string(int(r))}")
        return int(r)

    def unpacket_batch_begin(self, conns: Sequence[Connection], buffers: Sequence[RingBuffer]) -> int:
        """gevws_protocol_unpacket_batch_begin: stage and enqueue the pass, do not wait;
        returns the connections in it."""
        n = len(conns)
        cs = (ctypes.c_void_p * n)(*[c._p for c in conns])
        rs = (ctypes.c_void_p * n)(*[b._p for b in buffers])
        # the C side keeps the raw pointers until _end: hold the Python objects
        # too, so no Connection / RingBuffer is freed under a pass in flight
        self._pending = (cs, rs, list(conns), list(buffers))
        r = lib.gevws_protocol_unpacket_batch_begin(self._p, cs, rs, n)
        if r < 0:
            raise RuntimeError(f"unpacket_batch_begin: {status_string(int(r))}")
        return int(r)

    def unpacket_batch_end(self) -> int:
        """gevws_protocol_unpacket_batch_end: wait for the pass in flight and queue its frames."""
        r = lib.gevws_protocol_unpacket_batch_end(self._p)
        self._pending = None
        if r < 0:
            raise RuntimeError(f"unpacket_batch_end: {status_string(int(r))}")
        return int(r)

    def set_handler(self, policy: int) -> None:
        """gevws_protocol_set_handler: HandlerWrap.OnMessage on the device for
        every frame a pass decodes (GEVWS_HANDLER_*; -1 = off)."""
        st = lib.gevws_protocol_set_handler(self._p, int(policy))
        if st != OK:
            raise ValueError(f"set_handler({policy}): {status_string(st)}")

    def reply(self, c: Connection) -> Tuple[Optional[bytes], bool]:
        """gevws_protocol_reply: (reply wire bytes or None, ShutdownWrite) -- the
        device handler's answer for the frame unpacket() last returned on c."""
        out = _abi.U8P()
        n = ctypes.c_uint64()
        sh = ctypes.c_int()
        st = lib.gevws_protocol_reply(self._p, c._p, ctypes.byref(out), ctypes.byref(n), ctypes.byref(sh))
        if st != OK:
            raise RuntimeError(f"reply: {status_string(st)}")
        return (ctypes.string_at(out, n.value) if n.value else None), bool(sh.value)

    def set_service(self, on: bool) -> None:
        """gevws_protocol_set_service: zero-copy passes without a handler step
        go to the context's resident decode service (no launch call)."""
        st = lib.gevws_protocol_set_service(self._p, 1 if on else 0)
        if st != OK:
            raise RuntimeError(f"gevws_protocol_set_service: {status_string(st)}")

    def set_direct(self, on: bool) -> None:
        """gevws_protocol_set_direct: zero-copy passes without a handler step
        are written into the context's own AQL queue (no HIP launch call)."""
        st = lib.gevws_protocol_set_direct(self._p, 1 if on else 0)
        if st != OK:
            raise RuntimeError(f"gevws_protocol_set_direct: {status_string(st)}")

    def set_zero_copy_max(self, nbytes: int) -> None:
        """gevws_protocol_set_zero_copy_max: batched passes over at most
        `nbytes` of input run on mapped host memory with no copies (0 = never)."""
        lib.gevws_protocol_set_zero_copy_max(self._p, int(nbytes))

    def stats(self) -> dict:
        """Host-ingress counters (gevws_protocol_get_stats): device passes,
        connections and bytes staged, UnPacket calls answered by the host gate,
        passes run zero-copy."""
        s = _abi.ProtocolStats()
        lib.gevws_protocol_get_stats(self._p, ctypes.byref(s))
        return {k: int(getattr(s, k)) for k, _ in _abi.ProtocolStats._fields_}

    def timeline(self) -> dict:
        """Where the batched passes' time went (gevws_protocol_get_timeline):
        host ns per phase summed over the passes, and the one-launch kernels'
        GPU ns for passes answered by the completion flag."""
        t = _abi.ProtocolTimeline()
        lib.gevws_protocol_get_timeline(self._p, ctypes.byref(t))
        return {k: int(getattr(t, k)) for k, _ in _abi.ProtocolTimeline._fields_}

    def decode_host(self, segments: Sequence[Tuple[bytes, bytes]]):
        """gevws_decode_host_batch: [(first, end)] host segments per connection ->
        (frames, payload arena, conn_out, summary) as numpy arrays (the FFI form)."""
        n = len(segments)
        keep = []
        hc = (_abi.HostConn * max(n, 1))()
        total = 0
        for i, (a, b) in enumerate(segments):
            ba = np.frombuffer(a, np.uint8) if a else np.zeros(0, np.uint8)
            bb = np.frombuffer(b, np.uint8) if b else np.zeros(0, np.uint8)
            keep += [ba, bb]
            hc[i].seg0, hc[i].n0 = (ba.ctypes.data if ba.size else None), ba.size
            hc[i].seg1, hc[i].n1 = (bb.ctypes.data if bb.size else None), bb.size
            total += ba.size + bb.size
        max_frames = total // 2 + 1
        cap = total + 16 * max_frames + 16
        for _ in range(2):
            frames = np.zeros(max_frames, FRAME_DTYPE)
            payload = np.zeros(cap, np.uint8)
            cout = np.zeros(max(n, 1), CONN_OUT_DTYPE)
            s = _abi.Summary()
            r = lib.gevws_decode_host_batch(self._p, hc, n, frames.ctypes.data, max_frames, payload.ctypes.data,
                                            cap, cout.ctypes.data, ctypes.byref(s))
            if r == ERR_CAPACITY:
                max_frames, cap = max(s.frames, 1), max(s.payload_bytes, 16)
                continue
            if r < 0:
                raise RuntimeError(f"decode_host: {status_string(int(r))}")
            return frames[:s.frames], payload[:s.payload_bytes], cout[:n], s
        raise RuntimeError("decode_host: capacity retry failed")

    def packet(self, c: Connection, data: bytes) -> bytes:
        """Packet(c, data) -> data (protocol.go:67-69)."""
        return data


def handler_protocol(protocol: Protocol, c: Connection, buffer: RingBuffer,
                     on_message: Callable[[Connection, Optional[Header], bytes], Optional[bytes]]) -> List[bytes]:
    """Connection.handlerProtocol (connection.go:208-218): UnPacket until (nil, nil),
    handing each frame to on_message and collecting Packet'ed replies."""
    replies: List[bytes] = []
    ctx, data = protocol.unpacket(c, buffer)
    while ctx is not None or (data is not None and len(data) != 0):
        send = on_message(c, ctx, data)
        if send is not None:
            replies.append(protocol.packet(c, send))
        ctx, data = protocol.unpacket(c, buffer)
    return replies


__all__ = ["Engine", "Batch", "Comm", "RingBuffer", "Connection", "Protocol", "Header", "handler_protocol",
           "Upgrader", "RejectError", "HandshakeError", "HandshakeInfo", "accept_key", "HANDSHAKE", "ERR_HANDSHAKE",
           "status_string", "device_count", "lib", "FRAME_DTYPE", "CONN_OUT_DTYPE", "SUMMARY_DTYPE",
           "SYNTH_DTYPE", "OUT_FRAME_DTYPE", "OK", "NEED_MORE", "ERR_LEN_MSB", "ERR_CAPACITY", "ERR_INVALID", "ERR_DEVICE",
           "ERR_NOT_UPGRADED", "IN_PAD", "PAYLOAD_ALIGN", "TILE", "SUMMARY_UNORDERED"]
