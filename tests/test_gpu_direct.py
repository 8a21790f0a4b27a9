"""Direct dispatch (gevws_ctx_set_direct / gevws_decode_batch_post,
gev_amd/csrc/gevws_direct.cpp): a live pass written as one AQL packet into
the context's own HSA queue instead of launched through the HIP runtime.
Every pass is checked bit-exact against the C oracle (oracle/ref.decode_batch,
the restatement of plugins/websocket/protocol.go:34-84 + ws/read.go:19-84 +
ws/cipher.go:11-55), across both one-launch shapes, interleaved with launched
calls on the context's stream and on other streams (ordering both ways), and
through the Protocol and the live server."""
from __future__ import annotations

import numpy as np
import pytest

import gev_amd
from gev_amd import _abi
from tests._helpers import assert_matches_oracle, check_against_oracle, host_result, post_and_wait, random_batch

pytestmark = pytest.mark.gpu


@pytest.fixture
def direct(engine):
    import torch
    flag = gev_amd.PinnedArena(4096)
    engine.set_completion_flag(flag, 64)
    engine.set_direct(True)
    yield flag
    engine.set_direct(False)
    torch.cuda.synchronize()
    engine.set_completion_flag(None)
    flag.close()


def test_direct_passes_equal_oracle(engine, direct):
    """80 passes of 1..1 024 connections up to 128 KiB: both shapes, one slice
    and up to 32, all dispatched straight into the context's queue."""
    rng = np.random.default_rng(71)
    d0 = engine.direct_dispatches
    posted = 0
    for i in range(80):
        n = int(rng.choice([1, 5, 64, 200, 256, 300, 700, 1024]))
        a, conns = random_batch(rng, n, max_len=int(rng.choice([40, 120, 400])), frames=(1, 4))
        if a.size > _abi.ONE_LAUNCH_MAX_BYTES:
            continue
        got, _ = post_and_wait(engine, direct, a, conns)
        check_against_oracle(got, a, conns, f"pass {i}: {n} connections, {a.size} bytes")
        posted += 1
    assert posted >= 40
    assert engine.direct_dispatches - d0 == posted, (engine.direct_dispatches, d0, posted)


def test_direct_interleaved_with_launched_calls(engine, direct):
    """Direct passes alternating with launched decodes on the default stream
    (multi-kernel, sharing the context's scratch) and with one-launch calls on
    a torch stream: each side waits for the other, so every result is exact."""
    import torch
    rng = np.random.default_rng(72)
    dev = torch.device("cuda", engine.device)
    for i in range(6):
        a, conns = random_batch(rng, 150)
        got, _ = post_and_wait(engine, direct, a, conns)
        check_against_oracle(got, a, conns, f"direct {i}")
        a2, conns2 = random_batch(rng, 20, max_len=9000)  # past the one-launch limit: launched, multi-kernel
        assert_matches_oracle(engine, a2, conns2, f"launched {i}")
        # a direct pass, then at once a one-launch pass on another stream (same staging granules)
        a3, conns3 = random_batch(rng, 120)
        d_in = torch.zeros(a3.size + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
        d_in[: a3.size] = torch.from_numpy(a3).to(dev)
        d_c = torch.from_numpy(np.ascontiguousarray(conns3)).to(dev)
        mf, cap = a3.size // 2 + 1, a3.size * 9 + 64
        out = engine.alloc_batch(conns3.shape[0], mf, cap)
        d_in4 = torch.zeros(a.size + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
        d_in4[: a.size] = torch.from_numpy(a).to(dev)
        d_c4 = torch.from_numpy(np.ascontiguousarray(conns)).to(dev)
        mf4, cap4 = a.size // 2 + 1, a.size * 9 + 64
        out4 = engine.alloc_batch(conns.shape[0], mf4, cap4)
        torch.cuda.synchronize()
        engine.decode_post(d_in4, a.size, d_c4, conns.shape[0], out4, mf4, cap4)  # not waited for
        s1 = torch.cuda.Stream(dev)
        engine.decode_async(d_in, a3.size, d_c, conns3.shape[0], out, mf, cap, stream=s1)
        torch.cuda.synchronize()
        check_against_oracle(host_result(out4), a, conns, f"direct before stream {i}")
        check_against_oracle(host_result(out), a3, conns3, f"stream after direct {i}")


def test_direct_synchronize_and_off(engine, direct):
    """gevws_ctx_synchronize waits for direct passes; set_direct(False)
    launches again (the dispatch count stops)."""
    rng = np.random.default_rng(73)
    a, conns = random_batch(rng, 64)
    got, _ = post_and_wait(engine, direct, a, conns)
    engine.synchronize()
    check_against_oracle(got, a, conns, "direct")
    engine.set_direct(False)
    d0 = engine.direct_dispatches
    got, _ = post_and_wait(engine, direct, a, conns)
    check_against_oracle(got, a, conns, "launched")
    assert engine.direct_dispatches == d0


def test_protocol_zero_copy_passes_dispatched_direct(engine):
    """Protocol.set_direct: the 100-connection live shape's zero-copy passes
    go straight into the context's queue, are answered by the completion flag
    and deliver the oracle's frames."""
    from oracle import ws_oracle as wo
    rng = np.random.default_rng(74)
    proto = gev_amd.Protocol(engine)
    proto.set_direct(True)
    d0 = engine.direct_dispatches
    try:
        conns = [gev_amd.Connection() for _ in range(100)]
        rings, streams = [], []
        for c in conns:
            s = b"".join(wo.encode_frame(bytes(rng.integers(0, 256, int(rng.integers(1, 400)), dtype=np.uint8)), 1,
                                         True, 0, True, bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
                         for _ in range(2))
            r = gev_amd.RingBuffer(4096)
            r.write(s)
            rings.append(r)
            streams.append(s)
        for k in range(12):
            assert proto.unpacket_batch(conns, rings) == 200
            for c, r, s in zip(conns, rings, streams):
                for fr in wo.decode_stream(s).frames:
                    h, data = proto.unpacket(c, r)
                    assert data == fr.payload
                r.write(s)
        st = proto.stats()
        assert st["signalled_passes"] == 12, st
        assert engine.direct_dispatches - d0 == 12
    finally:
        proto.set_direct(False)
        proto.close()


def test_direct_and_service_on_one_context(engine, direct):
    """Both forms on: posts go to the context's own queue; with direct off
    they go to the resident service (the direct passes drained first), and
    back again (the service instance stopped first).  Every pass exact."""
    rng = np.random.default_rng(75)
    engine.set_service(True)
    try:
        for round_ in range(3):
            for form in ("direct", "service"):
                engine.set_direct(form == "direct")
                d0, s0 = engine.direct_dispatches, engine.service_stats()["posts"]
                for i in range(4):
                    a, conns = random_batch(rng, int(rng.choice([10, 100, 250])), max_len=100, frames=(1, 3))
                    assert a.size <= _abi.ONE_LAUNCH_MAX_BYTES // 2  # (the service's narrow shape)
                    got, _ = post_and_wait(engine, direct, a, conns)
                    check_against_oracle(got, a, conns, f"{form} {round_}.{i}")
                moved = engine.direct_dispatches - d0, engine.service_stats()["posts"] - s0
                assert moved == ((4, 0) if form == "direct" else (0, 4)), (form, moved)
    finally:
        engine.set_service(False)
        engine.set_direct(True)  # (the fixture turns it off)
