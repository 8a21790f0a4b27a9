"""CPU oracle for the websocket HTTP upgrade.

TEST INFRASTRUCTURE ONLY -- imported by tests/ as the checker of the product's
handshake (gev_amd/csrc/handshake.cpp through include/gevws.h); never part of
the product path.

Restates, from the reference sources (read as text):
  * Upgrader.Upgrade             plugins/websocket/ws/ws.go:158-343
  * httpParseRequestLine/Version ws/http.go:77-124, httpParseHeaderLine http.go:126-138
  * httpWriteResponseUpgrade     ws/http.go:174-200, httpWriteResponseError http.go:202-270
  * initAcceptFromNonce          ws/nonce.go:23-39
  * asciiToInt/pow/bsplit3/btrim/canonicalizeHeaderKey  ws/util.go:9-89
  * error values                 ws/errors.go:25-79
Pinned by RFC 6455 §1.3 (accept key) and §1.2/§4.2.2 (example handshake).
Sec-WebSocket-Protocol / -Extensions scanning lives in github.com/gobwas/httphead
(v0.0.0-20180130184737-2c6c146eadee, go.mod:10, not vendored): restated from
RFC 7230's list grammar -- parity unpinned.
"""
from __future__ import annotations

import base64
import hashlib
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Tuple

MAGIC = b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"

HS_OK, HS_MALFORMED, HS_BAD_PROTOCOL, HS_BAD_METHOD = 0, 1, 2, 3
HS_BAD_HOST, HS_BAD_UPGRADE, HS_BAD_CONNECTION, HS_BAD_SEC_ACCEPT = 4, 5, 6, 7
HS_BAD_SEC_KEY, HS_BAD_SEC_VERSION, HS_UPGRADE_REQUIRED, HS_HOOK = 8, 9, 10, 11

# errors.go:25-79 -> (code, reason, header)
STD_ERRORS = {
    HS_MALFORMED: (400, "malformed HTTP request", b""),
    HS_BAD_PROTOCOL: (505, "handshake error: bad HTTP protocol version", b""),
    HS_BAD_METHOD: (405, "handshake error: bad HTTP request method", b""),
    HS_BAD_HOST: (400, 'handshake error: bad "Host" header', b""),
    HS_BAD_UPGRADE: (400, 'handshake error: bad "Upgrade" header', b""),
    HS_BAD_CONNECTION: (400, 'handshake error: bad "Connection" header', b""),
    HS_BAD_SEC_ACCEPT: (400, 'handshake error: bad "Sec-WebSocket-Accept" header', b""),
    HS_BAD_SEC_KEY: (400, 'handshake error: bad "Sec-WebSocket-Key" header', b""),
    HS_BAD_SEC_VERSION: (400, 'handshake error: bad "Sec-WebSocket-Version" header', b""),
    HS_UPGRADE_REQUIRED: (426, 'handshake error: bad "Sec-WebSocket-Version" header',
                          b"Sec-WebSocket-Version: 13\r\n"),
}

STATUS_TEXT = {101: "Switching Protocols", 400: "Bad Request", 403: "Forbidden", 404: "Not Found",
               405: "Method Not Allowed", 426: "Upgrade Required", 500: "Internal Server Error",
               503: "Service Unavailable", 505: "HTTP Version Not Supported"}


def accept_from_nonce(nonce: bytes) -> bytes:
    """nonce.go:23-39."""
    assert len(nonce) == 24
    return base64.b64encode(hashlib.sha1(nonce + MAGIC).digest())


class Reject(Exception):
    """RejectConnectionError (errors.go:81-129); plain=True models errors.New."""

    def __init__(self, reason: str, code: int = 0, header: bytes = b"", plain: bool = False):
        super().__init__(reason)
        self.reason, self.code, self.header, self.plain = reason, code, header, plain


@dataclass
class Hooks:
    protocol: Optional[Callable[[bytes], bool]] = None
    protocol_custom: Optional[Callable[[bytes], Tuple[bytes, bool]]] = None
    extension: Optional[Callable[[bytes, list], bool]] = None
    on_request: Optional[Callable[[bytes], None]] = None
    on_host: Optional[Callable[[bytes], None]] = None
    on_header: Optional[Callable[[bytes, bytes], None]] = None
    on_before_upgrade: Optional[Callable[[], Optional[bytes]]] = None


@dataclass
class Result:
    out: bytes = b""
    consumed: int = 0
    error: int = HS_OK
    reason: str = ""
    http_code: int = 0
    protocol: bytes = b""
    extensions: bytes = b""
    seen_keys: List[bytes] = field(default_factory=list)


# ---------------------------------------------------------------- util.go
def ascii_to_int(b: bytes) -> Optional[int]:
    if len(b) < 1:
        return None
    ret = 0
    for i, c in enumerate(b):
        if c & 0xF0 != 0x30:
            return None
        ret += (c & 0xF) * (10 ** (len(b) - i - 1))
    ret &= (1 << 64) - 1                       # Go int wraps at 64 bits
    return ret - (1 << 64) if ret >> 63 else ret


def bsplit3(b: bytes, sep: int):
    a = b.find(bytes([sep]))
    c = b[a + 1:].find(bytes([sep]))
    if a == -1 or c == -1:
        return b, b"", b""
    c += a + 1
    return b[:a], b[a + 1:c], b[c + 1:]


def btrim(b: bytes) -> bytes:
    return b.strip(b" \t")


def canonical(k: bytes) -> bytes:
    out, upper = bytearray(k), True
    for i, c in enumerate(k):
        if upper and 0x61 <= c <= 0x7A:
            out[i] = c - 32
        elif not upper and 0x41 <= c <= 0x5A:
            out[i] = c + 32
        upper = c == 0x2D
    return bytes(out)


def parse_version(b: bytes):
    if b == b"HTTP/1.0":
        return 1, 0
    if b == b"HTTP/1.1":
        return 1, 1
    if len(b) < 8 or b[:5] != b"HTTP/":
        return None
    v = b[5:]
    dot = v.find(b".")
    if dot == -1:
        return None
    ma, mi = ascii_to_int(v[:dot]), ascii_to_int(v[dot + 1:])
    if ma is None or mi is None:
        return None
    return ma, mi


# ---------------------------------------------------------------- httphead (unpinned)
_SEP = set(b'()<>@,;:\\"/[]?={}')


def _tchar(c: int) -> bool:
    return 32 < c < 127 and c not in _SEP


def scan_tokens(h: bytes, it) -> bool:
    parts, any_tok = h.split(b","), False
    for idx, raw in enumerate(parts):
        t = raw.strip(b" \t")
        if not t:
            continue
        if not all(_tchar(c) for c in t):
            return False
        any_tok = True
        if not it(t):
            return True
    return any_tok


def scan_options(h: bytes):
    """1#( token *( ";" token [ "=" ( token / quoted-string ) ] ) ) -> [(name, [(k, v|None)])] or None."""
    i, n, out = 0, len(h), []

    def ws():
        nonlocal i
        while i < n and h[i] in (0x20, 0x09):
            i += 1

    def token():
        nonlocal i
        s = i
        while i < n and _tchar(h[i]):
            i += 1
        return h[s:i] if i > s else None

    while True:
        ws()
        if i >= n:
            break
        if h[i] == 0x2C:
            i += 1
            continue
        name = token()
        if name is None:
            return None
        params = []
        ws()
        while i < n and h[i] == 0x3B:
            i += 1
            ws()
            k = token()
            if k is None:
                return None
            ws()
            v = None
            if i < n and h[i] == 0x3D:
                i += 1
                ws()
                if i < n and h[i] == 0x22:
                    i += 1
                    buf, closed = bytearray(), False
                    while i < n:
                        if h[i] == 0x5C and i + 1 < n:
                            buf.append(h[i + 1])
                            i += 2
                        elif h[i] == 0x22:
                            i += 1
                            closed = True
                            break
                        else:
                            buf.append(h[i])
                            i += 1
                    if not closed:
                        return None
                    v = bytes(buf)
                else:
                    v = token()
                    if v is None:
                        return None
                ws()
            params.append((k, v))
        out.append((name, params))
        if i < n and h[i] != 0x2C:
            return None
    return out or None


def write_options(opts) -> bytes:
    s = []
    for name, params in opts:
        t = name
        for k, v in params:
            t += b";" + k
            if v is not None:
                if v and all(_tchar(c) for c in v):
                    t += b"=" + v
                else:
                    t += b'="' + v.replace(b"\\", b"\\\\").replace(b'"', b'\\"') + b'"'
        s.append(t)
    return b", ".join(s)


# ---------------------------------------------------------------- responses
def _status_line(code: int) -> bytes:
    return (f"HTTP/1.1 {code} {STATUS_TEXT.get(code, '')}\r\n"
            "Content-Type: text/plain; charset=utf-8\r\n").encode()


def write_error(code: int, headers: bytes, reason: str) -> bytes:
    body = reason.encode()
    return _status_line(code) + headers + b"Content-Length: %d\r\n\r\n" % len(body) + body


def write_upgrade(nonce: bytes, protocol: bytes, extensions: bytes, headers: bytes) -> bytes:
    o = (b"HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
         b"Sec-WebSocket-Accept: " + accept_from_nonce(nonce) + b"\r\n")
    if protocol:
        o += b"Sec-WebSocket-Protocol: " + protocol + b"\r\n"
    if extensions:
        o += b"Sec-WebSocket-Extensions: " + extensions + b"\r\n"
    return o + headers + b"\r\n"


# ---------------------------------------------------------------- Upgrade
def upgrade(first: bytes, end: bytes, hooks: Optional[Hooks] = None, header: bytes = b"") -> Result:
    """Upgrader.Upgrade over a ring's PeekAll() segments (first, end)."""
    hooks = hooks or Hooks()
    r = Result()
    joined = first + end
    data = b""
    idx = first.find(b"\r\n\r\n")
    if idx == -1 and end:
        idx = end.find(b"\r\n\r\n")
    if idx != -1:
        data = joined[: idx + 4]         # in.Read(data): from the front of the ring
        r.consumed = idx + 4
    lines = data.split(b"\r\n")

    def silent(kind, reason=None):
        r.error = kind
        r.reason = reason if reason is not None else STD_ERRORS[kind][1]
        return r

    method, uri, proto = bsplit3(lines[0], 0x20)
    ver = parse_version(proto)
    if ver is None:
        return silent(HS_MALFORMED)
    if ver[0] != 1 or ver[1] < 1:
        return silent(HS_BAD_PROTOCOL)
    if method != b"GET":
        return silent(HS_BAD_METHOD)
    if hooks.on_request:
        try:
            hooks.on_request(uri)
        except Reject as e:
            return silent(HS_HOOK, e.reason)

    err: Optional[Tuple[int, int, str, bytes, bool]] = None   # kind, code, reason, header, reject?
    seen, nonce, exts = 0, bytes(24), []

    def std(kind):
        code, reason, hdr = STD_ERRORS[kind]
        return kind, code, reason, hdr, True

    def hook(e: Reject):
        return HS_HOOK, (0 if e.plain else e.code), e.reason, (b"" if e.plain else e.header), not e.plain

    for line in lines[1:]:
        if err is not None or len(line) == 0:
            break
        colon = line.find(b":")
        if colon == -1:
            err = std(HS_MALFORMED)
            break
        k, v = canonical(btrim(line[:colon])), btrim(line[colon + 1:])
        r.seen_keys.append(k)
        try:
            if k == b"Host":
                seen |= 1
                if hooks.on_host:
                    hooks.on_host(v)
            elif k == b"Upgrade":
                seen |= 2
                if v != b"websocket":
                    err = std(HS_BAD_UPGRADE)
            elif k == b"Connection":
                seen |= 4
                if v not in (b"Upgrade", b"upgrade"):
                    err = std(HS_BAD_CONNECTION)
            elif k == b"Sec-Websocket-Version":
                seen |= 8
                if v != b"13":
                    err = std(HS_UPGRADE_REQUIRED)
            elif k == b"Sec-Websocket-Key":
                seen |= 16
                if len(v) != 24:
                    err = std(HS_BAD_SEC_KEY)
                else:
                    nonce = v
            elif k == b"Sec-Websocket-Protocol":
                if not r.protocol and (hooks.protocol_custom or hooks.protocol):
                    if hooks.protocol_custom:
                        r.protocol, ok = hooks.protocol_custom(v)
                    else:
                        sel = []
                        ok = scan_tokens(v, lambda t: not (hooks.protocol(t) and not sel.append(t)))
                        if ok and sel:
                            r.protocol = sel[0]
                    if not ok:
                        err = std(HS_MALFORMED)
            elif k == b"Sec-Websocket-Extensions":
                if hooks.extension:
                    offered = scan_options(v)
                    if offered is None:
                        err = std(HS_MALFORMED)
                    else:
                        for name, params in offered:
                            if any(name == s[0] for s in exts):
                                continue
                            if hooks.extension(name, params):
                                exts.append((name, params))
                        r.extensions = write_options(exts)
            elif hooks.on_header:
                hooks.on_header(k, v)
        except Reject as e:
            err = hook(e)

    extra = b""
    if err is None and seen != 31:
        for bit, kind in ((1, HS_BAD_HOST), (2, HS_BAD_UPGRADE), (4, HS_BAD_CONNECTION), (8, HS_BAD_SEC_VERSION),
                          (16, HS_BAD_SEC_KEY)):
            if not seen & bit:
                err = std(kind)
                break
    elif err is None and hooks.on_before_upgrade:
        try:
            extra = hooks.on_before_upgrade() or b""
        except Reject as e:
            err = hook(e)
    if err is not None:
        kind, code, reason, hdr, is_reject = err
        if is_reject:
            extra = hdr
        code = code if (is_reject and code) else 500
        r.error, r.reason, r.http_code = kind, reason, code
        r.out = write_error(code, header + extra, reason)
        return r
    r.out = write_upgrade(nonce, r.protocol, r.extensions, header + extra)
    r.http_code = 101
    return r
