"""Property-based parity on the device (hypothesis, shrinking to a minimal
failing batch): the HIP decode equals the C oracle (oracle/ws_ref.c, the
restatement of read.go:19-84 + protocol.go:38-62 + connection.go:208-218)
bit-exactly on generated batches -- every length class, minimal and
non-minimal length forms, any RSV / opcode, masked and unmasked frames,
garbage tails -- through the one-launch path and, with it turned off
(GEVWS_TUNE_SMALL_BATCH = 0), the multi-kernel path; and the device
ws.Cipher (cipher.go:14-53) equals the bytewise one at any offset and
alignment.  Strategies: tests/test_properties.py."""
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
