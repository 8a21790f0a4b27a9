"""The resident decode service (gevws_ctx_set_service / gevws_decode_batch_post,
gev_amd/csrc/gevws_walk.hip section 3d): a live loop's passes posted to a
kernel kept on the context's stream instead of launched.  Every pass is
checked bit-exact against the C oracle (oracle/ref.decode_batch, the
restatement of plugins/websocket/protocol.go:34-84 + ws/read.go:19-84 +
ws/cipher.go:11-55); the tests also pin the instance's life cycle -- reused
across passes, ended by any launched call (the posted pass still runs), by
a stop, and replaced after its use window -- and the Protocol's zero-copy
passes through it."""
from __future__ import annotations

import time

import numpy as np
import pytest

import gev_amd
from gev_amd import _abi
from oracle import ws_oracle as wo
from tests._helpers import assert_matches_oracle, check_against_oracle, post_and_wait, random_batch

pytestmark = pytest.mark.gpu


@pytest.fixture
def service(engine):
    import torch
    flag = gev_amd.PinnedArena(4096)
    engine.set_completion_flag(flag, 64)
    engine.set_service(True)
    yield flag
    engine.set_service(False)
    torch.cuda.synchronize()
    engine.set_completion_flag(None)
    flag.close()


def test_service_passes_equal_oracle(engine, service):
    """60 posted passes of 1..256 connections (one slice, decoded by
    workgroup 0 alone, up to 32 slices staged by every workgroup), one
    instance for all of them."""
    rng = np.random.default_rng(61)
    s0 = engine.service_stats()
    for i in range(60):
        n = int(rng.choice([1, 3, 17, 100, 256]))
        a, conns = random_batch(rng, n, max_len=int(rng.choice([60, 300, 900])))
        if a.size > _abi.ONE_LAUNCH_MAX_BYTES // 2:
            continue
        got, _ = post_and_wait(engine, service, a, conns)
        check_against_oracle(got, a, conns, f"pass {i}: {n} connections, {a.size} bytes")
    s1 = engine.service_stats()
    assert s1["posts"] - s0["posts"] >= 40, (s0, s1)
    # one instance, replaced at most every 100 ms
    assert s1["launches"] - s0["launches"] <= 1 + (s1["posts"] - s0["posts"]) // 5, (s0, s1)


def test_service_edges(engine, service):
    """No connections; empty and truncated streams; a 64 KiB pass (the
    narrow shape's limit: 32 slices); errors per connection (MSB length)."""
    rng = np.random.default_rng(62)
    cases = [(np.zeros(0, np.uint8), np.zeros((0, 2), np.int64))]
    a, conns = random_batch(rng, 5)
    conns[2, 1] = 0
    conns[4, 1] -= 3  # a frame cut short: left for the next read
    cases.append((a, conns))
    big = wo.encode_frame(bytes(rng.integers(0, 256, 65536 - 64 - 14, dtype=np.uint8)), 2, True, 0, True, b"abcd")
    a = np.frombuffer(big, np.uint8).copy()
    cases.append((a, np.array([[0, a.size]], np.int64)))
    bad = bytes([0x82, 0xFF]) + b"\x80" + b"\0" * 7 + b"key!"
    a = np.frombuffer(bad + bad, np.uint8).copy()
    cases.append((a, np.array([[0, len(bad)], [len(bad), len(bad)]], np.int64)))
    for i, (a, conns) in enumerate(cases):
        got, _ = post_and_wait(engine, service, a, conns)
        if conns.shape[0]:
            check_against_oracle(got, a, conns, f"case {i}")
        else:
            assert int(got["summary"]["status"]) == 0 and int(got["summary"]["frames"]) == 0


def test_service_ends_for_launched_calls_and_relaunches(engine, service):
    """Posts interleaved with ordinary (launched) decodes on the same context:
    each launched call ends the live instance first and runs behind it, the
    next post starts a new one; a pass past the narrow shape (300
    connections) is launched, not posted; an explicit stop and a gap past the
    instance's use window each give a fresh instance.  All bit-exact."""
    rng = np.random.default_rng(63)
    s0 = engine.service_stats()
    posts = 0
    for i in range(8):
        a, conns = random_batch(rng, 40)
        got, _ = post_and_wait(engine, service, a, conns)
        check_against_oracle(got, a, conns, f"posted {i}")
        posts += 1
        a2, conns2 = random_batch(rng, 30, max_len=5000)
        assert_matches_oracle(engine, a2, conns2, f"launched {i}")
    s1 = engine.service_stats()
    assert s1["posts"] - s0["posts"] == posts and s1["launches"] - s0["launches"] == posts, (s0, s1)
    a, conns = random_batch(rng, 300, max_len=80)  # past 256 connections: the wide one-launch shape, launched
    got, _ = post_and_wait(engine, service, a, conns)
    check_against_oracle(got, a, conns, "300 connections")
    s2 = engine.service_stats()
    assert s2["posts"] == s1["posts"], (s1, s2)
    a, conns = random_batch(rng, 20)
    got, _ = post_and_wait(engine, service, a, conns)
    engine.service_stop()
    got2, _ = post_and_wait(engine, service, a, conns)
    check_against_oracle(got, a, conns, "before stop")
    check_against_oracle(got2, a, conns, "after stop")
    time.sleep(0.25)  # past the use window (100 ms) and the instance's life (200 ms)
    got3, _ = post_and_wait(engine, service, a, conns)
    check_against_oracle(got3, a, conns, "after 250 ms")
    s3 = engine.service_stats()
    assert s3["posts"] - s2["posts"] == 3 and s3["launches"] - s2["launches"] == 3, (s2, s3)


def test_service_off_launches(engine, service):
    """set_service(False): decode_post is the one-launch decode again."""
    rng = np.random.default_rng(64)
    engine.set_service(False)
    s0 = engine.service_stats()
    a, conns = random_batch(rng, 50)
    got, _ = post_and_wait(engine, service, a, conns)
    check_against_oracle(got, a, conns, "service off")
    assert engine.service_stats() == s0


def test_protocol_zero_copy_passes_through_the_service(engine):
    """Protocol.set_service: the 100-connection live shape's zero-copy passes
    are posted, answered by the completion flag, and deliver the oracle's
    frames; a pass with the device handler chained is launched as before."""
    rng = np.random.default_rng(65)
    proto = gev_amd.Protocol(engine)
    proto.set_service(True)
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
        assert st["service_passes"] == 12 and st["signalled_passes"] == 12 and st["service_misses"] == 0, st
        t = proto.timeline()
        assert t["passes"] == 12 and t["signalled"] == 12, t
    finally:
        proto.set_service(False)
        proto.close()
