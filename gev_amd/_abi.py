"""ctypes binding of gev_amd/libgevws.so (declared in include/gevws.h).

The product path has no CPU fallback: if the HIP library is missing this
module raises ImportError, and device calls raise when no GPU is present.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgevws.so")

# status codes (gevws.h)
OK = 0
NEED_MORE = 1
ERR_LEN_MSB = -1
ERR_CAPACITY = -2
ERR_INVALID = -3
ERR_DEVICE = -4
ERR_NOT_UPGRADED = -5
HANDSHAKE = 2
ERR_HANDSHAKE = -6

# handshake error kinds (GEVWS_HS_*)
HS_OK = 0
HS_MALFORMED_REQUEST = 1
HS_BAD_PROTOCOL = 2
HS_BAD_METHOD = 3
HS_BAD_HOST = 4
HS_BAD_UPGRADE = 5
HS_BAD_CONNECTION = 6
HS_BAD_SEC_ACCEPT = 7
HS_BAD_SEC_KEY = 8
HS_BAD_SEC_VERSION = 9
HS_UPGRADE_REQUIRED = 10
HS_HOOK = 11

OUT_PAD = 16
AUX_SLOT = 128
HANDLER_NONE = 0
HANDLER_ECHO_BINARY = 1
HANDLER_ECHO_TEXT = 2
TUNE_UNMASK_VARIANT = 1  # 0 = auto (v3 / v5 per batch), 1 = v5 for every batch, 2 = auto with contiguous v5 runs
TUNE_UNMASK_GRID = 2
TUNE_ENCODE_VARIANT = 3  # 0 = auto, 1 / 2 = one / two tiles a wave step, 3 / 4 / 5 = two tiles, run mode 0 / 1 / 2
TUNE_WALK_VARIANT = 4  # 0 = default, 1 = plain chain walk, 2 = no entry table, 3 = writer wave always
TUNE_SMALL_BATCH = 7  # one-launch decode up to this many input bytes (0 = never)
ONE_LAUNCH_MAX_BYTES = 128 * 1024  # GEVWS_ONE_LAUNCH_MAX_BYTES: TUNE_SMALL_BATCH's default and maximum
ONE_LAUNCH_MAX_CONNS = 1024  # GEVWS_ONE_LAUNCH_MAX_CONNS
TUNE_SPLIT_LANES = 8  # split header walk: lanes per connection (0 = auto, 1 = never, 2/4/8/16/32)
TUNE_RETIRED = (5, 6, 9, 10, 11, 12)  # round 1-3 measurement knobs, rejected
TUNE_SPLIT_MIN_BYTES = 13  # split walk: bytes per segment at least (default 16 384)
TUNE_SPLIT_LANES_PER_CU = 14  # split walk auto: lanes per CU at most (default 512)

IN_PAD = 64
MEM_DEFAULT, MEM_FINE, MEM_UNCACHED = 0, 1, 2  # gevws_device_alloc kinds
SUMMARY_UNORDERED = 1  # summary.flags: connection table not in increasing input order
PAYLOAD_ALIGN = 16
TILE = 4096


class Header(ctypes.Structure):
    """gevws_header == ws.Header (plugins/websocket/ws/frame.go:169-176)."""
    _fields_ = [("fin", ctypes.c_uint8), ("rsv", ctypes.c_uint8), ("opcode", ctypes.c_uint8),
                ("masked", ctypes.c_uint8), ("mask", ctypes.c_uint8 * 4), ("length", ctypes.c_int64)]

    def as_tuple(self):
        return (bool(self.fin), self.rsv, self.opcode, bool(self.masked), bytes(self.mask), self.length)

    def __repr__(self):
        return ("Header(fin=%s, rsv=%d, opcode=%d, masked=%s, mask=%s, length=%d)"
                % (bool(self.fin), self.rsv, self.opcode, bool(self.masked), bytes(self.mask).hex(),
                   self.length))


class ConnIn(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint64), ("len", ctypes.c_uint64)]


class Frame(ctypes.Structure):
    _fields_ = [("hdr", Header), ("payload_off", ctypes.c_uint64), ("src_off", ctypes.c_uint64)]


class ConnOut(ctypes.Structure):
    _fields_ = [("first_frame", ctypes.c_uint64), ("consumed", ctypes.c_uint64),
                ("payload_base", ctypes.c_uint64), ("nframes", ctypes.c_uint32), ("status", ctypes.c_int32)]


class Summary(ctypes.Structure):
    _fields_ = [("frames", ctypes.c_uint64), ("payload_bytes", ctypes.c_uint64),
                ("payload_len", ctypes.c_uint64), ("errors", ctypes.c_uint64), ("status", ctypes.c_int32),
                ("flags", ctypes.c_uint32), ("run_frames", ctypes.c_uint64), ("reserved", ctypes.c_uint64 * 2)]


ZERO_COPY_MAX_DEFAULT = 256 * 1024  # GEVWS_ZERO_COPY_MAX_DEFAULT


class ProtocolStats(ctypes.Structure):
    _fields_ = [("device_passes", ctypes.c_uint64), ("conns_staged", ctypes.c_uint64),
                ("bytes_staged", ctypes.c_uint64), ("gated", ctypes.c_uint64),
                ("zero_copy_passes", ctypes.c_uint64), ("handler_passes", ctypes.c_uint64),
                ("chained_handler_passes", ctypes.c_uint64), ("signalled_passes", ctypes.c_uint64),
                ("service_passes", ctypes.c_uint64), ("service_misses", ctypes.c_uint64)]


class ProtocolTimeline(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("passes", "signalled", "ns_select", "ns_stage", "ns_launch", "ns_wait",
                                             "ns_deliver", "ns_gpu_decode", "ns_gpu_handler", "ns_gpu_gap")]


class HostConn(ctypes.Structure):
    _fields_ = [("seg0", ctypes.c_void_p), ("n0", ctypes.c_uint64), ("seg1", ctypes.c_void_p),
                ("n1", ctypes.c_uint64)]


class SynthDesc(ctypes.Structure):
    _fields_ = [("hdr_off", ctypes.c_uint64), ("length", ctypes.c_uint64), ("mask", ctypes.c_uint32),
                ("b0", ctypes.c_uint8), ("len_form", ctypes.c_uint8), ("masked", ctypes.c_uint8),
                ("pad", ctypes.c_uint8)]


class Reject(ctypes.Structure):
    """gevws_reject: RejectConnectionError options (ws/errors.go:81-129)."""
    _fields_ = [("code", ctypes.c_int32), ("plain", ctypes.c_int32), ("reason", ctypes.c_void_p),
                ("reason_len", ctypes.c_uint64), ("header", ctypes.c_void_p), ("header_len", ctypes.c_uint64)]


class ExtParam(ctypes.Structure):
    _fields_ = [("key", ctypes.c_void_p), ("key_len", ctypes.c_uint64), ("value", ctypes.c_void_p),
                ("value_len", ctypes.c_uint64)]


_VP, _U64 = ctypes.c_void_p, ctypes.c_uint64
_PU64 = ctypes.POINTER(ctypes.c_uint64)
_PVP = ctypes.POINTER(ctypes.c_void_p)
_PREJ = ctypes.POINTER(Reject)
HOOK_PROTOCOL = ctypes.CFUNCTYPE(ctypes.c_int, _VP, _VP, _U64)
HOOK_PROTOCOL_CUSTOM = ctypes.CFUNCTYPE(ctypes.c_int, _VP, _VP, _VP, _U64, _PVP, _PU64)
HOOK_EXTENSION = ctypes.CFUNCTYPE(ctypes.c_int, _VP, _VP, _U64, ctypes.POINTER(ExtParam), ctypes.c_uint32)
HOOK_EXTENSION_CUSTOM = ctypes.CFUNCTYPE(ctypes.c_int, _VP, _VP, _VP, _U64, _VP, _U64, _PVP, _PU64)
HOOK_ON_VALUE = ctypes.CFUNCTYPE(ctypes.c_int, _VP, _VP, _VP, _U64, _PREJ)
HOOK_ON_HEADER = ctypes.CFUNCTYPE(ctypes.c_int, _VP, _VP, _VP, _U64, _VP, _U64, _PREJ)
HOOK_ON_BEFORE_UPGRADE = ctypes.CFUNCTYPE(ctypes.c_int, _VP, _VP, _PVP, _PU64, _PREJ)


class UpgraderHooks(ctypes.Structure):
    """gevws_upgrader_hooks: ws.Upgrader's function fields (ws/ws.go:51-153)."""
    _fields_ = [("user", ctypes.c_void_p), ("protocol", HOOK_PROTOCOL),
                ("protocol_custom", HOOK_PROTOCOL_CUSTOM), ("extension", HOOK_EXTENSION),
                ("extension_custom", HOOK_EXTENSION_CUSTOM), ("on_request", HOOK_ON_VALUE),
                ("on_host", HOOK_ON_VALUE), ("on_header", HOOK_ON_HEADER),
                ("on_before_upgrade", HOOK_ON_BEFORE_UPGRADE)]


class Handshake(ctypes.Structure):
    """gevws_handshake: ws.Handshake (ws/ws.go:40-47) + error."""
    _fields_ = [("protocol", ctypes.c_void_p), ("protocol_len", ctypes.c_uint64),
                ("extensions", ctypes.c_void_p), ("extensions_len", ctypes.c_uint64),
                ("error", ctypes.c_int32), ("http_code", ctypes.c_int32), ("reason", ctypes.c_char_p)]


assert ctypes.sizeof(Reject) == 40 and ctypes.sizeof(UpgraderHooks) == 72 and ctypes.sizeof(Handshake) == 48
assert ctypes.sizeof(Header) == 16 and ctypes.sizeof(Frame) == 32
assert ctypes.sizeof(ConnIn) == 16 and ctypes.sizeof(ConnOut) == 32
assert ctypes.sizeof(Summary) == 64 and ctypes.sizeof(SynthDesc) == 24

P = ctypes.c_void_p
U8P = ctypes.POINTER(ctypes.c_uint8)

# (name, restype, argtypes) for every symbol include/gevws.h declares.
SIGNATURES = {
    "gevws_abi_version": (ctypes.c_int, []),
    "gevws_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "gevws_device_count": (ctypes.c_int, []),
    "gevws_ctx_create": (P, [ctypes.c_int]),
    "gevws_ctx_destroy": (None, [P]),
    "gevws_ctx_device": (ctypes.c_int, [P]),
    "gevws_ctx_stream": (P, [P]),
    "gevws_ctx_order_after_last": (ctypes.c_int, [P, P]),
    "gevws_ctx_set_timeline_ticks": (ctypes.c_int, [P, P]),
    "gevws_ctx_set_timing": (ctypes.c_int, [P, ctypes.c_int]),
    "gevws_ctx_set_tuning": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int64]),
    "gevws_ctx_last_split_lanes": (ctypes.c_int, [P]),
    "gevws_ctx_last_split_fallbacks": (ctypes.c_int64, [P]),
    "gevws_ctx_last_unmask_grid": (ctypes.c_int, [P]),
    "gevws_tuning_name": (ctypes.c_char_p, [ctypes.c_int, ctypes.c_int64]),
    "gevws_ctx_timing": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_uint32)]),
    "gevws_decode_batch_async": (ctypes.c_int, [P, P, P, ctypes.c_uint64, P, ctypes.c_uint32, P,
                                                ctypes.c_uint64, P, ctypes.c_uint64, P, P]),
    "gevws_decode_batch": (ctypes.c_int, [P, P, P, ctypes.c_uint64, P, ctypes.c_uint32, P,
                                          ctypes.c_uint64, P, ctypes.c_uint64, P, ctypes.POINTER(Summary)]),
    "gevws_encode_batch_async": (ctypes.c_int, [P, P, P, ctypes.c_uint64, P, P, ctypes.c_uint64, P, P]),
    "gevws_encode_replies_async": (ctypes.c_int, [P, P, P, ctypes.c_uint64, P, P, P, ctypes.c_uint64, P, P]),
    "gevws_dispatch_decoded_async": (ctypes.c_int, [P, P, P, ctypes.c_uint64, P, ctypes.c_int, P, ctypes.c_uint64,
                                                    ctypes.c_uint64, P, P, P]),
    "gevws_ctx_set_completion_flag": (ctypes.c_int, [P, P]),
    "gevws_ctx_set_service": (ctypes.c_int, [P, ctypes.c_int]),
    "gevws_ctx_service_stop": (ctypes.c_int, [P]),
    "gevws_ctx_service_stats": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "gevws_ctx_set_direct": (ctypes.c_int, [P, ctypes.c_int]),
    "gevws_ctx_direct_dispatches": (ctypes.c_int64, [P]),
    "gevws_ctx_synchronize": (ctypes.c_int, [P]),
    "gevws_decode_batch_post": (ctypes.c_int, [P, P, ctypes.c_uint64, P, ctypes.c_uint32, P, ctypes.c_uint64, P,
                                               ctypes.c_uint64, P, P]),
    "gevws_ctx_completion_seq": (ctypes.c_int64, [P]),
    "gevws_handle_decoded_async": (ctypes.c_int, [P, P, P, ctypes.c_uint64, P, ctypes.c_int, P, ctypes.c_uint64,
                                                  ctypes.c_uint64, P, P, P, P, ctypes.c_uint64, P, P]),
    "gevws_dispatch_async": (ctypes.c_int, [P, P, P, ctypes.c_uint64, ctypes.c_int, P, ctypes.c_uint64,
                                            ctypes.c_uint64, P, P, P]),
    "gevws_cipher_async": (ctypes.c_int, [P, P, P, ctypes.c_uint64, P, ctypes.c_uint64]),
    "gevws_synth_async": (ctypes.c_int, [P, P, P, P, ctypes.c_uint64, ctypes.c_uint64]),
    "gevws_synth_verify_async": (ctypes.c_int, [P, P, P, ctypes.c_uint64, ctypes.c_uint64, P, P,
                                                ctypes.c_uint64, P]),
    "gevws_ring_new": (P, [ctypes.c_uint64]),
    "gevws_ring_free": (None, [P]),
    "gevws_ring_write": (ctypes.c_uint64, [P, P, ctypes.c_uint64]),
    "gevws_ring_length": (ctypes.c_uint64, [P]),
    "gevws_ring_capacity": (ctypes.c_uint64, [P]),
    "gevws_ring_peek_all": (None, [P, ctypes.POINTER(U8P), ctypes.POINTER(ctypes.c_uint64),
                                   ctypes.POINTER(U8P), ctypes.POINTER(ctypes.c_uint64)]),
    "gevws_ring_retrieve": (None, [P, ctypes.c_uint64]),
    "gevws_conn_new": (P, []),
    "gevws_conn_free": (None, [P]),
    "gevws_conn_set_upgraded": (None, [P, ctypes.c_int]),
    "gevws_conn_upgraded": (ctypes.c_int, [P]),
    "gevws_conn_pending": (ctypes.c_uint64, [P]),
    "gevws_protocol_new": (P, [P]),
    "gevws_protocol_free": (None, [P]),
    "gevws_protocol_unpacket": (ctypes.c_int, [P, P, P, ctypes.POINTER(Header), ctypes.POINTER(U8P),
                                               ctypes.POINTER(ctypes.c_uint64)]),
    "gevws_protocol_unpacket_batch": (ctypes.c_int64, [P, P, P, ctypes.c_uint32]),
    "gevws_protocol_unpacket_batch_begin": (ctypes.c_int64, [P, P, P, ctypes.c_uint32]),
    "gevws_protocol_unpacket_batch_end": (ctypes.c_int64, [P]),
    "gevws_protocol_packet": (U8P, [P, P, P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    "gevws_copy_async": (ctypes.c_int, [P, P, P, P, ctypes.c_uint64, ctypes.c_uint32]),
    "gevws_pinned_alloc": (ctypes.c_int, [ctypes.c_uint64, ctypes.POINTER(P), ctypes.POINTER(P)]),
    "gevws_pinned_free": (ctypes.c_int, [P]),
    "gevws_device_alloc": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(P)]),
    "gevws_device_free": (ctypes.c_int, [ctypes.c_int, P]),
    "gevws_upgrader_new": (P, []),
    "gevws_upgrader_free": (None, [P]),
    "gevws_upgrader_set_header": (None, [P, P, ctypes.c_uint64]),
    "gevws_upgrader_set_hooks": (None, [P, ctypes.POINTER(UpgraderHooks)]),
    "gevws_upgrader_upgrade": (ctypes.c_int, [P, P, P, ctypes.POINTER(U8P), ctypes.POINTER(ctypes.c_uint64),
                                              ctypes.POINTER(Handshake)]),
    "gevws_conn_handshake": (ctypes.c_int, [P, ctypes.POINTER(Handshake)]),
    "gevws_handshake_error_string": (ctypes.c_char_p, [ctypes.c_int]),
    "gevws_accept_key": (None, [P, P]),
    "gevws_protocol_set_upgrader": (None, [P, P]),
    "gevws_decode_host_stream": (ctypes.c_int64, [P, P, ctypes.c_uint64, P, ctypes.c_uint64, P, ctypes.c_uint64,
                                                  P, ctypes.c_uint64, P, ctypes.POINTER(Summary)]),
    "gevws_parse_header": (ctypes.c_int, [P, ctypes.c_uint64, ctypes.POINTER(Header), ctypes.POINTER(ctypes.c_uint32)]),
    "gevws_parse_header_ring": (ctypes.c_int, [P, ctypes.c_uint64, P, ctypes.c_uint64, ctypes.POINTER(Header),
                                               ctypes.POINTER(ctypes.c_uint32)]),
    "gevws_cipher": (None, [P, ctypes.c_uint64, P, ctypes.c_uint64]),
    "gevws_protocol_get_stats": (None, [P, ctypes.POINTER(ProtocolStats)]),
    "gevws_protocol_get_timeline": (None, [P, ctypes.POINTER(ProtocolTimeline)]),
    "gevws_protocol_set_zero_copy_max": (None, [P, ctypes.c_uint64]),
    "gevws_protocol_set_service": (ctypes.c_int, [P, ctypes.c_int]),
    "gevws_protocol_set_direct": (ctypes.c_int, [P, ctypes.c_int]),
    "gevws_protocol_set_handler": (ctypes.c_int, [P, ctypes.c_int]),
    "gevws_comm_create": (P, [ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "gevws_comm_destroy": (None, [P]),
    "gevws_comm_size": (ctypes.c_int, [P]),
    "gevws_counts_allreduce_async": (ctypes.c_int, [P, ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P)]),
    "gevws_counts_allreduce": (ctypes.c_int, [P, ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P),
                                              ctypes.POINTER(ctypes.c_int64)]),
    "gevws_protocol_reply": (ctypes.c_int, [P, P, ctypes.POINTER(U8P), ctypes.POINTER(ctypes.c_uint64),
                                            ctypes.POINTER(ctypes.c_int)]),
    "gevws_decode_host_batch": (ctypes.c_int64, [P, P, ctypes.c_uint32, P, ctypes.c_uint64, P, ctypes.c_uint64,
                                                 P, ctypes.POINTER(Summary)]),
}


def _share_torch_hip_runtime() -> None:
    """torch wheels bundle their own libamdhip64.so.7; import torch first so
    that libgevws.so's libamdhip64.so.7 dependency binds to that same runtime
    (one HIP runtime per process: device pointers, streams and events are
    shared with torch).  Without torch, /opt/rocm's runtime is used."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    _share_torch_hip_runtime()
    if not os.path.exists(path):
        raise ImportError(
            f"gev_amd: HIP library {path} is missing -- build it first "
            "(python -c 'import __graft_entry__ as g; g.build()'); there is no CPU fallback")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib
