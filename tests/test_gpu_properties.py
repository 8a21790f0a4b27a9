"""Property-based parity on the device (hypothesis, shrinking to a minimal
failing batch): the HIP decode equals the C oracle (oracle/ws_ref.c, the
restatement of read.go:19-84 + protocol.go:38-62 + connection.go:208-218)
bit-exactly on generated batches -- every length class, minimal and
non-minimal length forms, any RSV / opcode, masked and unmasked frames,
garbage tails -- through the one-launch path and, with it turned off
(GEVWS_TUNE_SMALL_BATCH = 0), the multi-kernel path; and the device
ws.Cipher (cipher.go:14-53) equals the bytewise one at any offset and
alignment; the device encode (FrameToBytes) equals the C oracle's on
generated records.  Stream strategies: tests/test_properties.py."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import gev_amd
from gev_amd import _abi
from oracle import ws_oracle as wo
from tests._helpers import assert_matches_oracle, pack_streams
from tests.test_properties import streams

pytestmark = pytest.mark.gpu

SETTINGS = settings(max_examples=300, deadline=None,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


@SETTINGS
@given(st.lists(streams, min_size=1, max_size=8), st.booleans())
def test_device_decode_equals_oracle(engine, ss, one_launch):
    arena, conns = pack_streams(ss)
    engine.set_tuning(_abi.TUNE_SMALL_BATCH, 65536 if one_launch else 0)
    try:
        assert_matches_oracle(engine, arena, conns, f"one_launch={one_launch}")
    finally:
        engine.set_tuning(_abi.TUNE_SMALL_BATCH, 65536)


@SETTINGS
@given(st.binary(min_size=1, max_size=600), st.binary(min_size=4, max_size=4), st.integers(0, 1 << 20),
       st.integers(0, 15))
def test_device_cipher_equals_bytewise(engine, payload, mask, offset, align):
    import torch
    buf = torch.zeros(align + len(payload) + 64, dtype=torch.uint8, device=torch.device("cuda", engine.device))
    buf[align:align + len(payload)] = torch.from_numpy(np.frombuffer(payload, np.uint8).copy()).to(buf.device)
    engine.cipher_(buf, mask, offset, nbytes=len(payload), byte_offset=align)
    torch.cuda.synchronize()
    want = bytearray(payload)
    wo.cipher_bytewise(want, mask, offset)
    got = buf.cpu().numpy().tobytes()
    assert got[align:align + len(payload)] == bytes(want)
    assert got[:align] == b"\0" * align and got[align + len(payload):] == b"\0" * 64


@st.composite
def out_frames(draw):
    """Records for the encode (OUT_FRAME_DTYPE) over one payload arena: any
    FIN / RSV / opcode / MASK bit and key, lengths across the 7-, 16- and
    64-bit forms, payloads at any alignment (overlapping ones too)."""
    n = draw(st.integers(0, 24))
    lens = [draw(st.one_of(st.integers(0, 300), st.sampled_from([125, 126, 65535, 65536]), st.integers(0, 70000)))
            for _ in range(n)]
    arena_len = sum(lens) + 64
    fr = np.zeros(n, gev_amd.OUT_FRAME_DTYPE)
    for i, L in enumerate(lens):
        fr[i]["fin"] = draw(st.integers(0, 1))
        fr[i]["rsv"] = draw(st.integers(0, 7))
        fr[i]["opcode"] = draw(st.integers(0, 15))
        fr[i]["masked"] = draw(st.integers(0, 1))
        fr[i]["mask"] = np.frombuffer(draw(st.binary(min_size=4, max_size=4)), np.uint8)
        fr[i]["length"] = L
        fr[i]["payload_len"] = L
        fr[i]["payload_off"] = draw(st.integers(0, arena_len - L))
    seed = draw(st.integers(0, 2**32 - 1))
    payload = np.random.default_rng(seed).integers(0, 256, arena_len, dtype=np.uint8)
    return fr, payload


@settings(max_examples=150, deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture,
                                 HealthCheck.data_too_large])
@given(out_frames())
def test_device_encode_equals_oracle(engine, case):
    """FrameToBytes (frame.go:274-278 over write.go:48-84) on the device equals
    oracle/ws_ref.c's encode: wire bytes and every frame's wire offset."""
    import torch
    from oracle import ref
    fr, payload = case
    d_pay = torch.from_numpy(np.concatenate([payload, np.zeros(16, np.uint8)])).to(torch.device("cuda", engine.device))
    wire, off = engine.encode(fr, d_pay)
    want, woff = ref.encode_batch(fr, payload)
    assert np.array_equal(wire.cpu().numpy(), want)
    assert np.array_equal(off, woff)
