"""CPU oracle for the WebSocket frame-decode / payload-unmask hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``gev_amd/`` may import, call or link
this module: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker.

This is a plain-Python restatement of the reference (Allenxuxu/gev, Go) written
from its semantics; no reference source is copied.  Each function cites the
reference file:line it follows (paths relative to the reference root).

Parity pinning
--------------
The reference has no golden vectors or known-answer tests for this path
 and cannot be built here (no Go toolchain).  The oracle is
pinned by:

* RFC 6455 §5.7 known-answer frames (see ``RFC6455_KATS`` below), which the
  reference's header layout (read.go:19-84) and XOR (cipher.go:14-53) must
  reproduce;
* properties: ``cipher`` (the Go word-loop transliteration) equals the bytewise
  definition for every offset mod 4 and every length; involution; chunk/offset
  composition;
* the C restatement ``oracle/ws_ref.c`` agreeing with this module.

Edge cases that depend on the un-vendored ``github.com/Allenxuxu/ringbuffer
v0.0.11`` are **parity unpinned**; the oracle
takes the RFC-correct choice (NEED_MORE) and the golden fixtures exclude them.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

# Status codes (mirror include/gevws.h).
OK = 0
NEED_MORE = 1          # ws.ErrHeaderNotReady / completeness gate failed -> (nil, nil)
ERR_LEN_MSB = -1       # ws.ErrHeaderLengthMSB (read.go:12-16, 71-73)

# Opcodes, frame.go:14-25.
OP_CONTINUATION = 0x0
OP_TEXT = 0x1
OP_BINARY = 0x2
OP_CLOSE = 0x8
OP_PING = 0x9
OP_PONG = 0xA

# remain maps mask position [0,4) to bytes processed one by one (cipher.go:56).
_REMAIN = (0, 3, 2, 1)


@dataclass
class Header:
    """ws.Header, frame.go:169-176: {Fin bool; Rsv byte; OpCode; Masked bool;
    Mask [4]byte; Length int64} -- 16 bytes in Go's layout."""
    fin: bool = False
    rsv: int = 0
    opcode: int = 0
    masked: bool = False
    mask: bytes = b"\x00\x00\x00\x00"
    length: int = 0

    def pack(self) -> bytes:
        """Byte image identical to the Go struct / gevws_header (offsets 0,1,2,3,4..7,8..15)."""
        return struct.pack("<BBBB4sq", int(self.fin), self.rsv, self.opcode,
                           int(self.masked), self.mask, self.length)

    @staticmethod
    def unpack(b: bytes) -> "Header":
        fin, rsv, op, masked, mask, length = struct.unpack("<BBBB4sq", b)
        return Header(bool(fin), rsv, op, bool(masked), mask, length)


# --------------------------------------------------------------------------- cipher
def cipher_bytewise(payload: bytearray, mask: bytes, offset: int = 0) -> None:
    """Definition of the XOR unmask: p[i] ^= mask[(offset+i) % 4]
    (RFC 6455 §5.3; cipher.go:16-21 is exactly this loop for n < 8)."""
    for i in range(len(payload)):
        payload[i] ^= mask[(offset + i) % 4]


def cipher(payload: bytearray, mask: bytes, offset: int = 0) -> None:
    """Transliteration of ws.Cipher, cipher.go:14-53, in place.

    n < 8: bytewise (cipher.go:16-21).  Otherwise ``ln = remain[offset%4]`` head
    bytes and ``rn = (n-ln)%8`` tail bytes bytewise (cipher.go:24-36), then the
    body as native-endian uint64 words XORed with ``m<<32|m`` where ``m`` is the
    native-endian uint32 of the mask (cipher.go:42-51).  Python's ``int.from_bytes
    (..., 'little')`` stands in for x86 native endianness; the algorithm is
    endianness-agnostic by construction (cipher.go:38-41).
    """
    n = len(payload)
    if n < 8:
        for i in range(n):
            payload[i] ^= mask[(offset + i) % 4]
        return
    mpos = offset % 4
    ln = _REMAIN[mpos]
    rn = (n - ln) % 8
    for i in range(ln):
        payload[i] ^= mask[(mpos + i) % 4]
    for i in range(n - rn, n):
        payload[i] ^= mask[(mpos + i) % 4]
    m = int.from_bytes(mask, "little")
    m2 = (m << 32) | m
    words = (n - ln - rn) >> 3
    for i in range(words):
        s = ln + (i << 3)
        v = int.from_bytes(payload[s:s + 8], "little") ^ m2
        payload[s:s + 8] = v.to_bytes(8, "little")


def cipher_np(payload, mask: bytes, offset: int = 0):
    """numpy form of the bytewise definition for medium sizes (returns a new array)."""
    import numpy as np
    p = np.frombuffer(bytes(payload), dtype=np.uint8) if not isinstance(payload, np.ndarray) else payload
    n = p.shape[0]
    key = np.frombuffer(mask, dtype=np.uint8)
    idx = (np.arange(n, dtype=np.int64) + offset) & 3
    return p ^ key[idx]


# --------------------------------------------------------------------------- header
def read_header(buf, pos: int = 0, avail: Optional[int] = None) -> Tuple[int, Optional[Header], int]:
    """ws.VirtualReadHeader, read.go:19-84, over a linear view of the ring.

    Returns ``(status, header, header_len)``.

    * ``avail < 6`` -> NEED_MORE even for complete 2..5-byte unmasked frames
      (read.go:20-23; Appendix A P1).
    * byte0: FIN = bit7, RSV = (b0 & 0x70) >> 4, opcode = b0 & 0x0F (read.go:29-31).
    * byte1: MASK = bit7 -> +4 extra; len7 = b1 & 0x7F; 126 -> +2 BE16;
      127 -> +8 BE64 (read.go:33-49).
    * 127-form with the length MSB set -> ERR_LEN_MSB (read.go:69-73).
    * The mask is the last 4 extra bytes (read.go:78-81).
    * No validation of RSV, reserved opcodes, control-frame size or minimal
      length encoding (Appendix A P5).
    * U1 (avail >= 6 but < header length): the reference reads stale scratch
      bytes (ringbuffer-dependent, unpinned); the oracle answers NEED_MORE.
    """
    if avail is None:
        avail = len(buf) - pos
    if avail < 6:
        return NEED_MORE, None, 0
    b0 = buf[pos]
    b1 = buf[pos + 1]
    h = Header()
    h.fin = (b0 & 0x80) != 0
    h.rsv = (b0 & 0x70) >> 4
    h.opcode = b0 & 0x0F
    extra = 0
    if b1 & 0x80:
        h.masked = True
        extra += 4
    len7 = b1 & 0x7F
    if len7 < 126:
        h.length = len7
    elif len7 == 126:
        extra += 2
    else:
        extra += 8
    hlen = 2 + extra
    if extra == 0:
        return OK, h, hlen
    if avail < hlen:               # U1: unpinned -> RFC-correct NEED_MORE
        return NEED_MORE, None, 0
    e = pos + 2
    if len7 == 126:
        h.length = (buf[e] << 8) | buf[e + 1]
        e += 2
    elif len7 == 127:
        if buf[e] & 0x80:
            return ERR_LEN_MSB, None, 0
        h.length = int.from_bytes(bytes(buf[e:e + 8]), "big")
        e += 8
    if h.masked:
        h.mask = bytes(buf[e:e + 4])
    return OK, h, hlen


# --------------------------------------------------------------------------- unpacket
@dataclass
class Frame:
    header: Header
    payload: bytes
    header_len: int
    stream_pos: int  # offset of the frame's first header byte in the connection stream


def unpacket(buf, pos: int = 0) -> Tuple[int, Optional[Frame]]:
    """One call of websocket.(*Protocol).UnPacket's decode branch,
    plugins/websocket/protocol.go:38-62, on a linear view starting at ``pos``.

    Header (read_header) -> completeness gate ``VirtualLength() >= Length``
    (protocol.go:47) -> fresh zero-filled slice of Length, filled from the ring
    (protocol.go:48-51) -> ``Cipher(payload, mask, 0)`` iff Masked
    (protocol.go:53-55; mask phase restarts at 0 per frame, Appendix A P7).
    Incomplete -> NEED_MORE with nothing consumed (protocol.go:59-61).
    """
    avail = len(buf) - pos
    st, h, hlen = read_header(buf, pos, avail)
    if st != OK:
        return st, None
    if avail - hlen < h.length:
        return NEED_MORE, None
    start = pos + hlen
    payload = bytearray(bytes(buf[start:start + h.length]))
    if h.masked:
        cipher(payload, h.mask, 0)
    return OK, Frame(h, bytes(payload), hlen, pos)


@dataclass
class StreamResult:
    frames: List[Frame] = field(default_factory=list)
    consumed: int = 0
    status: int = OK       # OK (stopped on NEED_MORE) or ERR_LEN_MSB (connection poisoned)


def decode_stream(buf) -> StreamResult:
    """Connection.handlerProtocol, connection.go:208-218: call UnPacket until it
    returns (nil, nil), preserving stream order.  A header error stops the loop
    too (protocol.go:41-45 returns (nil, nil)); ERR_LEN_MSB poisons the stream
    (Appendix A P9/U3)."""
    res = StreamResult()
    pos = 0
    while True:
        st, fr = unpacket(buf, pos)
        if st != OK:
            res.status = OK if st == NEED_MORE else st
            break
        res.frames.append(fr)
        pos += fr.header_len + fr.header.length
    res.consumed = pos
    return res


# --------------------------------------------------------------------------- outbound encode (§8f row 1)
def write_header_go(h: Header) -> bytes:
    """ws.WriteHeader, write.go:48-84, byte for byte -- including Go's byte
    arithmetic: ``bts[0] |= h.Rsv << 4`` keeps the low 8 bits, ``OpCode`` is
    OR-ed as a whole byte, and any Length <= 125 (negative ones too) is written
    as ``byte(h.Length)``.  The MASK bit and key follow the length
    (write.go:78-81); the payload is NOT masked by FrameToBytes."""
    bts = bytearray(14)
    if h.fin:
        bts[0] |= 0x80
    bts[0] |= (h.rsv << 4) & 0xFF
    bts[0] |= h.opcode & 0xFF
    L = h.length
    if L <= 125:
        bts[1] = L & 0xFF
        n = 2
    elif L <= 0xFFFF:
        bts[1] = 126
        bts[2:4] = L.to_bytes(2, "big")
        n = 4
    else:
        bts[1] = 127
        bts[2:10] = L.to_bytes(8, "big")
        n = 10
    if h.masked:
        bts[1] |= 0x80
        bts[n:n + 4] = h.mask
        n += 4
    return bytes(bts[:n])


def frame_to_bytes(h: Header, payload: bytes) -> bytes:
    """ws.FrameToBytes, frame.go:274-278: WriteHeader(&f.Header) + payload."""
    return write_header_go(h) + bytes(payload)


def new_frame(op: int, fin: bool, p: bytes) -> Tuple[Header, bytes]:
    """ws.NewFrame, frame.go:193-203 (NewBinaryFrame/NewTextFrame/NewPongFrame...)."""
    return Header(fin=fin, rsv=0, opcode=op, masked=False, mask=b"\x00" * 4, length=len(p)), p


# --------------------------------------------------------------------------- control-frame dispatch (§8f row 2)
MAX_CONTROL_PAYLOAD = 125                      # frame.go:9-10
STATUS_PROTOCOL_ERROR = 1002                   # frame.go:80-83
_PROTOCOL_DEFINED = {1000, 1001, 1002, 1003, 1007, 1008, 1009, 1010, 1011, 1005, 1006, 1015}  # frame.go:130-147
_PROTOCOL_RESERVED = {1005, 1006, 1015}        # frame.go:151-160
ERR_NOT_IN_USE = b"status code is not in use"              # errors.go:17-21
ERR_APP_LEVEL = b"status code is only application level"
ERR_NO_MEANING = b"status code has no meaning yet"
ERR_UNKNOWN = b"status code is not defined in spec"
ERR_INVALID_UTF8 = b"invalid utf8 sequence in close reason"

HANDLER_NONE = 0          # the user's WSHandler returns nothing
HANDLER_ECHO_BINARY = 1   # benchmarks/websocket/server.go:22-29 (MessageBinary, data)
HANDLER_ECHO_TEXT = 2     # example/websocket OnMessage shape (MessageText, data)


def utf8_valid(b: bytes) -> bool:
    """unicode/utf8.ValidString: strict UTF-8 (no surrogates, no overlongs, <= U+10FFFF)."""
    try:
        b.decode("utf-8", errors="strict")
        return True
    except UnicodeDecodeError:
        return False


def parse_close_frame_data(payload: bytes) -> Tuple[int, bytes]:
    """ws.ParseCloseFrameData, read.go:89-102."""
    if len(payload) < 2:
        return 0, b""
    return int.from_bytes(payload[:2], "big"), payload[2:]


def check_close_frame_data(code: int, reason: bytes) -> Optional[bytes]:
    """util.CheckCloseFrameData, util/util.go:65-85 (switch order kept)."""
    if 0 <= code <= 999:
        return ERR_NOT_IN_USE
    if code in _PROTOCOL_RESERVED:
        return ERR_APP_LEVEL
    if code == 1004:
        return ERR_NO_MEANING
    if 1000 <= code <= 2999 and code not in _PROTOCOL_DEFINED:
        return ERR_UNKNOWN
    if not utf8_valid(reason):
        return ERR_INVALID_UTF8
    return None


def new_close_frame_body(code: int, reason: bytes) -> bytes:
    """ws.NewCloseFrameBody, frame.go:251-259: min(2+len, 125) bytes, reason
    cropped to 123."""
    n = min(2 + len(reason), MAX_CONTROL_PAYLOAD)
    crop = min(MAX_CONTROL_PAYLOAD - 2, len(reason))
    return (code.to_bytes(2, "big") + reason[:crop])[:n]


def handle_close(h: Header, payload: bytes) -> bytes:
    """util.HandleClose, util/util.go:27-46."""
    if h.length == 0:
        return write_header_go(Header(fin=True, opcode=OP_CLOSE))
    code, reason = parse_close_frame_data(payload)
    err = check_close_frame_data(code, reason)
    if err is not None:
        body = new_close_frame_body(STATUS_PROTOCOL_ERROR, err)
    else:
        body = new_close_frame_body(code, reason)
    return frame_to_bytes(*new_frame(OP_CLOSE, True, body))


def on_message(h: Header, payload: bytes, policy: int) -> Tuple[Optional[bytes], bool]:
    """HandlerWrap.OnMessage, plugins/websocket/wrap.go:38-90, for a decoded frame.
    Returns (reply bytes or None, ShutdownWrite called).  Control frames:
    close -> HandleClose + ShutdownWrite (wrap.go:51-56); ping -> pong with the
    same payload (util.go:49-51); pong -> PING with the same payload (util.go:54-56,
    the reference's quirk); other control opcodes -> no reply.  Data frames go
    to the user handler (here an echo policy); an empty reply sends nothing
    (wrap.go:72)."""
    op = h.opcode
    if op & 0x8:
        if op == OP_CLOSE:
            return handle_close(h, payload), True
        if op == OP_PING:
            return frame_to_bytes(*new_frame(OP_PONG, True, payload)), False
        if op == OP_PONG:
            return frame_to_bytes(*new_frame(OP_PING, True, payload)), False
        return None, False
    if policy == HANDLER_NONE or len(payload) == 0:
        return None, False
    op_out = OP_BINARY if policy == HANDLER_ECHO_BINARY else OP_TEXT
    return frame_to_bytes(*new_frame(op_out, True, payload)), False


# --------------------------------------------------------------------------- encoder (fixtures)
def write_header(fin: bool, rsv: int, opcode: int, length: int, masked: bool,
                 mask: bytes = b"\x00\x00\x00\x00", len_form: Optional[int] = None) -> bytes:
    """Header serialisation following ws.WriteHeader, write.go:48-84 (minimal
    length form: <=125 -> 7-bit, <=0xFFFF -> 126+BE16, else 127+BE64) plus the
    client MASK bit and key (write.go:78-81).  ``len_form`` forces a
    non-minimal encoding (7, 16 or 64) to build Appendix A P5 cases."""
    b0 = (0x80 if fin else 0) | ((rsv & 7) << 4) | (opcode & 0x0F)
    if len_form is None:
        len_form = 7 if length <= 125 else (16 if length <= 0xFFFF else 64)
    if len_form == 7:
        assert length <= 125
        out = bytearray([b0, length])
    elif len_form == 16:
        assert length <= 0xFFFF
        out = bytearray([b0, 126]) + length.to_bytes(2, "big")
    else:
        out = bytearray([b0, 127]) + length.to_bytes(8, "big")
    if masked:
        out[1] |= 0x80
        out += mask
    return bytes(out)


def encode_frame(payload: bytes, opcode: int = OP_BINARY, fin: bool = True, rsv: int = 0,
                 masked: bool = True, mask: bytes = b"\x00\x00\x00\x00",
                 len_form: Optional[int] = None) -> bytes:
    """A complete client->server frame: header + payload XORed with the key."""
    hdr = write_header(fin, rsv, opcode, len(payload), masked, mask, len_form)
    body = bytearray(payload)
    if masked:
        cipher_bytewise(body, mask, 0)
    return hdr + bytes(body)


# RFC 6455 §5.7 known-answer frames (external KATs; see module docstring).
RFC6455_KATS = [
    # (wire bytes, fin, opcode, masked, mask, payload)
    (bytes.fromhex("810548656c6c6f"), True, OP_TEXT, False, b"\x00" * 4, b"Hello"),
    (bytes.fromhex("818537fa213d7f9f4d5158"), True, OP_TEXT, True, bytes.fromhex("37fa213d"), b"Hello"),
    (bytes.fromhex("010348656c"), False, OP_TEXT, False, b"\x00" * 4, b"Hel"),
    (bytes.fromhex("80026c6f"), True, OP_CONTINUATION, False, b"\x00" * 4, b"lo"),
    (bytes.fromhex("890548656c6c6f"), True, OP_PING, False, b"\x00" * 4, b"Hello"),
    (bytes.fromhex("8a8537fa213d7f9f4d5158"), True, OP_PONG, True, bytes.fromhex("37fa213d"), b"Hello"),
]
# Header-only KATs (§5.7: 256-byte and 64 KiB unmasked binary messages).
RFC6455_HEADER_KATS = [
    (bytes.fromhex("827e0100"), True, OP_BINARY, False, 256, 4),
    (bytes.fromhex("827f0000000000010000"), True, OP_BINARY, False, 65536, 10),
]
