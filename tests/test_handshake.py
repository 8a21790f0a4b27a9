"""The websocket HTTP upgrade: the product's
Upgrader.Upgrade (gev_amd/csrc/handshake.cpp via include/gevws.h; host code, so
these run on the CPU) against the oracle restatement (oracle/ws_handshake.py)
and RFC 6455's worked examples.  Reference: plugins/websocket/ws/ws.go:158-343,
http.go, nonce.go, util.go, errors.go."""
import random

import pytest

import gev_amd
from gev_amd import _abi
from oracle import ws_handshake as wh

RFC_KEY = b"dGhlIHNhbXBsZSBub25jZQ=="          # RFC 6455 §1.3
RFC_ACCEPT = b"s3pPLMBiTxaQ9kYGzzhZRbK+xOo="

RFC_REQUEST = (b"GET /chat HTTP/1.1\r\nHost: server.example.com\r\nUpgrade: websocket\r\n"
               b"Connection: Upgrade\r\nSec-WebSocket-Key: dGhlIHNhbXBsZSBub25jZQ==\r\n"
               b"Origin: http://example.com\r\nSec-WebSocket-Protocol: chat, superchat\r\n"
               b"Sec-WebSocket-Version: 13\r\n\r\n")
# golang.org/x/net/websocket's hybi client request, as the reference's own echo
# test sends it (example/websocket/wsserver_test.go:106, websocket.Dial)
XNET_REQUEST = (b"GET / HTTP/1.1\r\nHost: localhost:1834\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                b"Sec-WebSocket-Key: x3JJHMbDL1EzLkh9GBhXDw==\r\nOrigin: ws://localhost:1834\r\n"
                b"Sec-WebSocket-Version: 13\r\n\r\n")


def _ring_with(data: bytes, wrap_at=None, size=None):
    """A RingBuffer holding `data`; with wrap_at, its first segment ends after
    wrap_at bytes (the write wraps round the end of the buffer)."""
    if wrap_at is None:
        r = gev_amd.RingBuffer(size or max(len(data), 1))
        r.write(data)
        return r
    size = len(data) + 7
    r = gev_amd.RingBuffer(size)
    pre = size - wrap_at
    r.write(b"\0" * pre)
    r.retrieve(pre - 1)          # keep one byte: emptying the ring rewinds it
    r.write(data)
    r.retrieve(1)
    first, end = r.peek_all()
    assert len(first) == wrap_at and first + end == data
    return r


def _both(data: bytes, product_upgrader=None, oracle_hooks=None, header=b"", wrap_at=None):
    r = _ring_with(data, wrap_at)
    first, end = r.peek_all()
    want = wh.upgrade(first, end, oracle_hooks, header)
    u = product_upgrader or gev_amd.Upgrader(header=header)
    c = gev_amd.Connection(upgraded=False)
    out, info, err = u.upgrade(c, r)
    assert out == want.out
    assert info.error == want.error and info.reason == want.reason
    assert info.http_code == want.http_code
    assert info.protocol == want.protocol and info.extensions == want.extensions
    assert r.length() == len(data) - want.consumed
    assert (err is None) == (want.error == wh.HS_OK)
    return out, info, want


def test_accept_key_rfc6455_kat():
    assert wh.accept_from_nonce(RFC_KEY) == RFC_ACCEPT
    assert gev_amd.accept_key(RFC_KEY) == RFC_ACCEPT


def test_accept_key_random_nonces():
    rng = random.Random(5)
    alphabet = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/="
    for _ in range(300):
        nonce = bytes(rng.choice(alphabet) for _ in range(24))
        assert gev_amd.accept_key(nonce) == wh.accept_from_nonce(nonce)


def test_rfc6455_example_handshake():
    out, info, _ = _both(RFC_REQUEST + b"\x81\x85")
    assert out == (b"HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                   b"Sec-WebSocket-Accept: s3pPLMBiTxaQ9kYGzzhZRbK+xOo=\r\n\r\n")
    assert info.error == _abi.HS_OK and info.protocol == b""      # no Protocol hook: nothing selected


def test_reference_test_client_request():
    out, info, _ = _both(XNET_REQUEST)
    assert out.startswith(b"HTTP/1.1 101 Switching Protocols\r\n") and info.http_code == 101
    assert b"Sec-WebSocket-Accept: " + wh.accept_from_nonce(b"x3JJHMbDL1EzLkh9GBhXDw==") in out


@pytest.mark.parametrize("wrap_at", [5, 40, 120, len(XNET_REQUEST) - 3, len(XNET_REQUEST) - 1])
def test_request_split_across_ring_segments(wrap_at):
    """ws.go:178-192: the head is found in the first segment, or in the second
    alone (then index+4 bytes are read from the ring's front: fewer than the
    head); a terminator straddling the segments is never found."""
    _both(XNET_REQUEST + b"\x82\x80abcd", wrap_at=wrap_at)


def test_incomplete_head_reads_nothing():
    for cut in (0, 1, 16, len(RFC_REQUEST) - 1):
        out, info, want = _both(RFC_REQUEST[:cut])
        assert out == b"" and info.error == _abi.HS_MALFORMED_REQUEST and want.consumed == 0


def _req(lines, method=b"GET", uri=b"/", proto=b"HTTP/1.1"):
    return method + b" " + uri + b" " + proto + b"\r\n" + b"".join(l + b"\r\n" for l in lines) + b"\r\n"


GOOD = [b"Host: h", b"Upgrade: websocket", b"Connection: Upgrade", b"Sec-WebSocket-Version: 13",
        b"Sec-WebSocket-Key: " + RFC_KEY]


@pytest.mark.parametrize("case,kind,code", [
    (_req(GOOD, proto=b"HTTP/1.0"), _abi.HS_BAD_PROTOCOL, 0),
    (_req(GOOD, proto=b"HTTP/2.1"), _abi.HS_BAD_PROTOCOL, 0),
    (_req(GOOD, proto=b"HTTP/1.:"), _abi.HS_OK, 101),          # ':' counts as digit 10 (util.go:17)
    (_req(GOOD, proto=b"HTTP/x.1"), _abi.HS_MALFORMED_REQUEST, 0),
    (_req(GOOD, method=b"POST"), _abi.HS_BAD_METHOD, 0),
    (b"GET /\r\n" + b"".join(l + b"\r\n" for l in GOOD) + b"\r\n", _abi.HS_MALFORMED_REQUEST, 0),
    (_req(GOOD[1:]), _abi.HS_BAD_HOST, 400),
    (_req(GOOD[:1] + GOOD[2:]), _abi.HS_BAD_UPGRADE, 400),
    (_req(GOOD[:2] + GOOD[3:]), _abi.HS_BAD_CONNECTION, 400),
    (_req(GOOD[:3] + GOOD[4:]), _abi.HS_BAD_SEC_VERSION, 400),
    (_req(GOOD[:4]), _abi.HS_BAD_SEC_KEY, 400),
    (_req([b"Host: h"]), _abi.HS_BAD_UPGRADE, 400),
    (_req(GOOD[:1] + [b"Upgrade: WebSocket"] + GOOD[2:]), _abi.HS_BAD_UPGRADE, 400),  # case-sensitive
    (_req(GOOD[:2] + [b"Connection: keep-alive, Upgrade"] + GOOD[3:]), _abi.HS_BAD_CONNECTION, 400),
    (_req(GOOD[:2] + [b"Connection: upgrade"] + GOOD[3:]), _abi.HS_OK, 101),
    (_req(GOOD[:3] + [b"Sec-WebSocket-Version: 8"] + GOOD[4:]), _abi.HS_UPGRADE_REQUIRED, 426),
    (_req(GOOD[:4] + [b"Sec-WebSocket-Key: short"]), _abi.HS_BAD_SEC_KEY, 400),
    (_req(GOOD[:2] + [b"no colon here"] + GOOD[2:]), _abi.HS_MALFORMED_REQUEST, 400),
    (_req([b"  hOsT \t:  h ", b"UPGRADE:websocket", b"connection:Upgrade", b"sec-websocket-version: 13",
           b"SEC-WEBSOCKET-KEY:" + RFC_KEY]), _abi.HS_OK, 101),
])
def test_request_checks(case, kind, code):
    out, info, _ = _both(case)
    assert info.error == kind and info.http_code == code


def test_error_response_bytes():
    out, _, _ = _both(_req(GOOD[:3] + [b"Sec-WebSocket-Version: 7"] + GOOD[4:]))
    reason = b'handshake error: bad "Sec-WebSocket-Version" header'
    assert out == (b"HTTP/1.1 426 Upgrade Required\r\nContent-Type: text/plain; charset=utf-8\r\n"
                   b"Sec-WebSocket-Version: 13\r\nContent-Length: %d\r\n\r\n" % len(reason) + reason)


def test_upgrader_header_in_every_response():
    h = b"X-Server: gev\r\n"
    out, _, _ = _both(_req(GOOD), header=h)
    assert out.endswith(h + b"\r\n")
    out, _, _ = _both(_req(GOOD[1:]), header=h)
    assert h in out and out.startswith(b"HTTP/1.1 400 Bad Request")


def test_hooks_reject_and_accept():
    seen = []

    def on_request(c, uri):
        assert isinstance(c, gev_amd.Connection)      # hooks get the gev.Connection
        seen.append(("uri", uri))
        if uri == b"/deny":
            raise gev_amd.RejectError("nope", 403)

    def on_host(c, host):
        if host == b"bad":
            raise gev_amd.RejectError("bad host", 403, b"X-Why: host\r\n")

    def on_header(c, k, v):
        seen.append((k, v))
        if k == b"X-Fail":
            raise ValueError("plain failure")

    def on_before_upgrade(c):
        return b"X-Extra: 1\r\n"

    u = gev_amd.Upgrader(on_request=on_request, on_host=on_host, on_header=on_header,
                         on_before_upgrade=on_before_upgrade)

    def o_request(uri):
        if uri == b"/deny":
            raise wh.Reject("nope", 403)

    def o_host(h):
        if h == b"bad":
            raise wh.Reject("bad host", 403, b"X-Why: host\r\n")

    def o_header(k, v):
        if k == b"X-Fail":
            raise wh.Reject("plain failure", plain=True)

    hooks = wh.Hooks(on_request=o_request, on_host=o_host, on_header=o_header,
                     on_before_upgrade=lambda: b"X-Extra: 1\r\n")
    # OnRequest rejection: no response (ws.go:222-229)
    out, info, _ = _both(_req(GOOD, uri=b"/deny"), u, hooks)
    assert out == b"" and info.error == _abi.HS_HOOK and info.reason == "nope"
    # OnHost rejection with status + header
    out, info, _ = _both(_req([b"Host: bad"] + GOOD[1:]), u, hooks)
    assert out.startswith(b"HTTP/1.1 403 Forbidden\r\n") and b"X-Why: host\r\n" in out
    # a plain error from OnHeader -> 500 (ws.go:325-333)
    out, info, _ = _both(_req(GOOD[:2] + [b"x-fail: 1"] + GOOD[2:]), u, hooks)
    assert out.startswith(b"HTTP/1.1 500 Internal Server Error\r\n") and out.endswith(b"plain failure")
    # success: OnBeforeUpgrade's header, OnHeader saw canonical keys
    seen.clear()
    out, info, _ = _both(_req(GOOD + [b"origin: x", b"x-custom-thing: y"]), u, hooks)
    assert info.http_code == 101 and out.endswith(b"X-Extra: 1\r\n\r\n")
    assert (b"Origin", b"x") in seen and (b"X-Custom-Thing", b"y") in seen


def test_before_upgrade_reject():
    u = gev_amd.Upgrader(on_before_upgrade=lambda c: (_ for _ in ()).throw(gev_amd.RejectError("later", 503)))

    def o_bu():
        raise wh.Reject("later", 503)
    out, info, _ = _both(_req(GOOD), u, wh.Hooks(on_before_upgrade=o_bu))
    assert out.startswith(b"HTTP/1.1 503 Service Unavailable\r\n") and info.http_code == 503


def test_subprotocol_selection():
    """Upgrader.Protocol: the first offered token the hook accepts (ws.go:282-292).
    Token scanning is gobwas/httphead's: parity unpinned beyond RFC 7230 lists."""
    pick = {b"superchat"}
    u = gev_amd.Upgrader(protocol=lambda t: t in pick)
    hooks = wh.Hooks(protocol=lambda t: t in pick)
    for offer, want in [(b"chat, superchat", b"superchat"), (b"superchat", b"superchat"), (b"chat", b""),
                        (b" chat ,superchat ", b"superchat"), (b"chat super", None), (b"", None), (b",", None)]:
        out, info, _ = _both(_req(GOOD + [b"Sec-WebSocket-Protocol: " + offer]), u, hooks)
        if want is None:
            assert info.error == _abi.HS_MALFORMED_REQUEST
        else:
            assert info.protocol == want
            assert (b"Sec-WebSocket-Protocol: " + want + b"\r\n" in out) == bool(want)
    # ProtocolCustom takes precedence
    u2 = gev_amd.Upgrader(protocol_custom=lambda c, v: (v.split(b",")[-1].strip(), True))
    h2 = wh.Hooks(protocol_custom=lambda v: (v.split(b",")[-1].strip(), True))
    out, info, _ = _both(_req(GOOD + [b"Sec-WebSocket-Protocol: a, b"]), u2, h2)
    assert info.protocol == b"b"


def test_extension_selection():
    """Upgrader.Extension with SelectUnique (http.go:156-162): parity unpinned
    (gobwas/httphead is not vendored), checked against the RFC 7230 restatement."""
    def accept(name, params):
        return name == b"permessage-deflate"
    u = gev_amd.Upgrader(extension=lambda name, params: accept(name, params))
    hooks = wh.Hooks(extension=accept)
    offer = b"permessage-deflate; client_max_window_bits, permessage-deflate; server_no_context_takeover, x-foo"
    out, info, _ = _both(_req(GOOD + [b"Sec-WebSocket-Extensions: " + offer]), u, hooks)
    assert info.extensions == b"permessage-deflate;client_max_window_bits"
    assert b"Sec-WebSocket-Extensions: permessage-deflate;client_max_window_bits\r\n" in out
    out, info, _ = _both(_req(GOOD + [b'Sec-WebSocket-Extensions: permessage-deflate; a="x y"']), u, hooks)
    assert info.extensions == b'permessage-deflate;a="x y"'
    out, info, _ = _both(_req(GOOD + [b"Sec-WebSocket-Extensions: ;bad"]), u, hooks)
    assert info.error == _abi.HS_MALFORMED_REQUEST


def test_randomised_requests_match_oracle():
    """Mutated header sets, orders, casings and values: product == oracle byte for byte."""
    rng = random.Random(1234)
    variants = {
        b"Host": [b"h", b"example.com:80", b""],
        b"Upgrade": [b"websocket", b"WebSocket", b"h2c"],
        b"Connection": [b"Upgrade", b"upgrade", b"close"],
        b"Sec-WebSocket-Version": [b"13", b"8", b" 13 "],
        b"Sec-WebSocket-Key": [RFC_KEY, b"x3JJHMbDL1EzLkh9GBhXDw==", b"tooshort", b"A" * 25],
    }
    for _ in range(600):
        lines = []
        for k, vals in variants.items():
            if rng.random() < 0.93:
                kk = bytes(c ^ 0x20 if (0x41 <= (c | 0x20) <= 0x7A and rng.random() < 0.2) else c for c in k)
                lines.append(kk + rng.choice([b": ", b":", b" :\t"]) + rng.choice(vals))
        for _ in range(rng.randrange(3)):
            lines.append(rng.choice([b"Origin: o", b"User-Agent: t", b"X: y", b"broken", b"Cookie: a=b"]))
        rng.shuffle(lines)
        req = _req(lines, method=rng.choice([b"GET"] * 8 + [b"PUT"]),
                   proto=rng.choice([b"HTTP/1.1"] * 8 + [b"HTTP/1.0", b"HTTP/1.2", b"HTTP/11"]))
        tail = bytes(rng.randrange(256) for _ in range(rng.randrange(8)))
        wrap = rng.choice([None, None, rng.randrange(1, len(req) + len(tail))])
        _both(req + tail, wrap_at=wrap)
