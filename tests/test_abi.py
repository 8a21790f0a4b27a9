"""CPU checks of the drop-in boundary: libgevws.so loads and exports every
symbol include/gevws.h declares, the ABI structs have the reference layouts,
and the host-side mirror (ring buffer, connection context) behaves like the
ringbuffer/gev calls it replaces.  No device compute is called here."""
import ctypes
import os
import re

import numpy as np
import pytest

import gev_amd
from gev_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "gevws.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gevws_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_what_binding_binds():
    assert declared_symbols() == sorted(_abi.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_abi.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_no_cpp_symbols_leak():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True).stdout
    exported = [ln.split()[-1] for ln in out.splitlines() if " T " in ln]
    assert exported and all(s.startswith("gevws_") for s in exported), [s for s in exported if not s.startswith("gevws_")]


def test_struct_layouts_match_reference():
    # ws.Header (frame.go:169-176): Fin@0 Rsv@1 OpCode@2 Masked@3 Mask@4..7 Length@8..15
    H = _abi.Header
    assert ctypes.sizeof(H) == 16
    assert [getattr(H, f).offset for f in ("fin", "rsv", "opcode", "masked", "mask", "length")] == [0, 1, 2, 3, 4, 8]
    assert gev_amd.FRAME_DTYPE.itemsize == ctypes.sizeof(_abi.Frame) == 32
    assert gev_amd.CONN_OUT_DTYPE.itemsize == ctypes.sizeof(_abi.ConnOut) == 32
    for f in ("first_frame", "consumed", "payload_base", "nframes", "status"):
        assert gev_amd.CONN_OUT_DTYPE.fields[f][1] == getattr(_abi.ConnOut, f).offset
    for f in ("hdr_off", "length", "mask", "b0", "len_form", "masked"):
        assert gev_amd.SYNTH_DTYPE.fields[f][1] == getattr(_abi.SynthDesc, f).offset


def test_status_strings_and_version():
    assert gev_amd.lib.gevws_abi_version() == 3  # round 6: gevws_protocol_stats grew
    assert gev_amd.status_string(gev_amd.NEED_MORE) == "header error: not enough"  # read.go:15
    assert gev_amd.status_string(gev_amd.ERR_LEN_MSB) == "header error: the most significant bit must be 0"


def test_fails_loudly_without_device():
    if gev_amd.device_count() > 0:
        pytest.skip("a device is present")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        gev_amd.Engine(0)
    assert gev_amd.lib.gevws_ctx_create(0) is None


def test_missing_library_is_an_import_error(tmp_path):
    with pytest.raises(ImportError, match="no CPU fallback"):
        _abi.load(str(tmp_path / "nope.so"))


def test_ring_buffer_write_peek_retrieve_wrap():
    r = gev_amd.RingBuffer(8)
    assert r.length() == 0 and r.is_empty()
    r.write(b"abcdef")
    r.retrieve(4)
    r.write(b"ghij")            # wraps: "ef" | "ghij"
    assert r.length() == 6
    first, end = r.peek_all()
    assert first + end == b"efghij" and first == b"efgh" and end == b"ij"
    r.write(b"0123456789")      # grows, keeps order
    assert r.capacity() >= 16
    assert b"".join(r.peek_all()) == b"efghij0123456789"
    r.retrieve(100)
    assert r.is_empty() and r.peek_all() == (b"", b"")


def test_default_protocol_unpacket_ring_fixture():
    """TestDefaultProtocol_UnPacket (protocol_test.go:13-31), the reference's one
    ring-buffer fixture, literally: ringbuffer.New(4), Write("1234") -> 4,
    Peek(2) + Retrieve(2), Write("ab") -> 2 (wraps into the freed front, no
    growth), then DefaultProtocol.UnPacket (protocol.go:19-39: PeekAll, join the
    two segments, RetrieveAll) returns "34ab" and Length() is 0."""
    r = gev_amd.RingBuffer(4)
    assert r.write(b"1234") == 4
    assert r.capacity() == 4 and r.length() == 4
    r.retrieve(2)  # (Peek(2) reads without consuming)
    assert r.write(b"ab") == 2
    assert r.capacity() == 4  # the write wrapped instead of growing
    s, e = r.peek_all()
    assert (s, e) == (b"34", b"ab")  # two segments: len(e) > 0 takes the userBuffer join
    data = s + e
    r.retrieve(len(s) + len(e))  # RetrieveAll
    assert data == b"34ab"
    assert r.length() == 0


def test_ring_buffer_random_against_bytes_model():
    rng = np.random.default_rng(3)
    r = gev_amd.RingBuffer(16)
    model = b""
    for _ in range(2000):
        if rng.random() < 0.55:
            d = bytes(rng.integers(0, 256, int(rng.integers(0, 70)), dtype=np.uint8))
            r.write(d)
            model += d
        else:
            k = int(rng.integers(0, 80))
            r.retrieve(k)
            model = model[k:]
        assert r.length() == len(model)
        assert b"".join(r.peek_all()) == model


def test_connection_context_keys():
    c = gev_amd.Connection(upgraded=False)
    assert not c.upgraded and c.pending() == 0
    c.set_upgraded(True)
    assert c.upgraded


def test_packet_is_identity():
    assert gev_amd.Protocol.packet(None, None, b"xyz") == b"xyz"
