"""Split-stream decode (gevws_ctx_set_unmask_stream): the header walk, scan and
record pass on one stream, the unmask on another, two batches in flight on
CU-masked streams -- the server loop of connection.go:208-218 with batch k+1's
walk beside batch k's unmask.  Results must be the oracle's, bit-exact, and
every in-flight slot must verify."""
import ctypes

import numpy as np
import pytest
import torch

import gev_amd
from oracle import ref
from tests._helpers import host_result, pack_streams, random_stream

pytestmark = pytest.mark.gpu


def _masked_streams(dev_index, front_cus=32):
    ncu = torch.cuda.get_device_properties(dev_index).multi_processor_count
    fm, bm = gev_amd.cu_split_masks(ncu, front_cus)
    return gev_amd.CuStream(dev_index, fm), gev_amd.CuStream(dev_index, bm), ncu


def test_cu_masked_streams_report_their_cus(engine):
    front, back, ncu = _masked_streams(engine.device)
    assert front.cus == 32 and back.cus == ncu - 32
    with pytest.raises(ValueError):
        gev_amd.cu_split_masks(ncu, 12)


def test_split_stream_decode_matches_oracle(engine):
    front, back, _ = _masked_streams(engine.device)
    dev = torch.device("cuda", engine.device)
    rng = np.random.default_rng(77)
    engine.set_unmask_stream(back)
    try:
        for it in range(4):
            n = int(rng.integers(300, 900))  # above the one-launch small-batch path
            arena, conns = pack_streams([random_stream(rng, int(rng.integers(0, 40))) for _ in range(n)])
            a = np.frombuffer(arena, np.uint8).copy()
            want = ref.decode_batch(a, conns[:, 0], conns[:, 1])
            d_in = torch.zeros(a.size + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
            d_in[: a.size] = torch.from_numpy(a).to(dev)
            d_conns = torch.from_numpy(conns.copy()).to(dev)
            nf = max(int(want["frames"].shape[0]), 1)
            cap = max(int(want["payload"].size), 16)
            out = engine.alloc_batch(n, nf, cap)
            torch.cuda.synchronize()
            engine.decode_async(d_in, a.size, d_conns, n, out, nf, cap, stream=front)
            engine.order_after_last(torch.cuda.current_stream(dev))
            got = host_result(out)
            assert int(got["summary"]["status"]) == 0
            assert got["frames"][: want["frames"].shape[0]].tobytes() == want["frames"].tobytes(), it
            assert np.array_equal(got["payload"][: want["payload"].size], want["payload"]), it
            assert np.array_equal(got["conn_out"]["consumed"], want["conn_consumed"]), it
    finally:
        engine.set_unmask_stream(None)


def test_two_batches_in_flight_on_masked_streams():
    """Two contexts share the front and unmask streams; 6 steps alternate
    between them with no host synchronisation; every slot's last batch is the
    generator's plaintext on every byte."""
    from gev_amd import workloads as w
    front, back, _ = _masked_streams(0)
    dev = torch.device("cuda", 0)
    lay = w.config_c4(total_payload=256 << 20, n_conns=2048, seed=5)
    arena = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    arena[lay.arena_bytes:] = 0
    desc = torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev)
    conns = torch.from_numpy(lay.conns.copy()).to(dev)
    engs = [gev_amd.Engine(0) for _ in range(2)]
    engs[0].synth(arena, desc, lay.n_frames, lay.seed)
    torch.cuda.synchronize()
    outs = [e.alloc_batch(lay.n_conns, lay.n_frames, lay.payload_padded) for e in engs]
    for e in engs:
        e.set_unmask_stream(back)
    for i in range(6):
        k = i % 2
        engs[k].decode_async(arena, lay.arena_bytes, conns, lay.n_conns, outs[k], lay.n_frames,
                             lay.payload_padded, stream=front)
    torch.cuda.synchronize()
    for k, e in enumerate(engs):
        mism = torch.zeros(1, dtype=torch.int64, device=dev)
        e.verify(desc, lay.n_frames, lay.seed, outs[k], mism)
        torch.cuda.synchronize()
        s = outs[k].summary_host()
        assert int(mism.item()) == 0, k
        assert int(s["frames"]) == lay.n_frames and int(s["payload_len"]) == lay.payload_len
        e.set_unmask_stream(None)
        e.close()


@pytest.mark.parametrize("kind", ["fine", "uncached"])
def test_decode_from_fine_and_uncached_input(kind):
    """The input arena in fine-grained or uncached device memory
    (gevws_device_alloc, the bench's --input-mem): the same records and
    payload bytes as from default memory, and every byte the generator's."""
    from gev_amd import workloads as w
    dev = torch.device("cuda", 0)
    eng = gev_amd.Engine(0)
    lay = w.config_c4(total_payload=64 << 20, n_conns=512, seed=9)
    desc = torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev)
    conns = torch.from_numpy(lay.conns.copy()).to(dev)
    base = torch.zeros(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    arena = gev_amd.DeviceArena(0, lay.arena_bytes + gev_amd.IN_PAD,
                                gev_amd.MEM_FINE if kind == "fine" else gev_amd.MEM_UNCACHED)
    outs = []
    for a in (base, arena):
        eng.synth(a, desc, lay.n_frames, lay.seed)
        out = eng.alloc_batch(lay.n_conns, lay.n_frames, lay.payload_padded)
        eng.decode_async(a, lay.arena_bytes, conns, lay.n_conns, out, lay.n_frames, lay.payload_padded)
        mism = torch.zeros(1, dtype=torch.int64, device=dev)
        eng.verify(desc, lay.n_frames, lay.seed, out, mism)
        torch.cuda.synchronize()
        assert int(mism.item()) == 0
        outs.append(out)
    assert torch.equal(outs[0].frames, outs[1].frames)
    assert torch.equal(outs[0].payload[:lay.payload_padded], outs[1].payload[:lay.payload_padded])
    arena.close()
    eng.close()


def test_sync_decode_waits_for_the_unmask_stream(engine):
    """gevws_decode_batch (the synchronous form) with an unmask stream set
    returns only after the unmask: checked on a third stream with no device
    synchronisation in between, every payload byte is the generator's."""
    from gev_amd import workloads as w
    front, back, _ = _masked_streams(engine.device)
    dev = torch.device("cuda", engine.device)
    lay = w.config_c4(total_payload=256 << 20, n_conns=2048, seed=11)
    arena = torch.zeros(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    desc = torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev)
    conns = torch.from_numpy(lay.conns.copy()).to(dev)
    engine.synth(arena, desc, lay.n_frames, lay.seed)
    out = engine.alloc_batch(lay.n_conns, lay.n_frames, lay.payload_padded)
    mism = torch.zeros(1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    from gev_amd import _abi
    h_sum = _abi.Summary()
    engine.set_unmask_stream(back)
    try:
        st = gev_amd.lib.gevws_decode_batch(engine._ctx, front.cuda_stream, arena.data_ptr(), lay.arena_bytes,
                                            conns.data_ptr(), lay.n_conns, out.frames.data_ptr(), lay.n_frames,
                                            out.payload.data_ptr(), lay.payload_padded, out.conn_out.data_ptr(),
                                            ctypes.byref(h_sum))
        assert st == gev_amd.OK
        assert int(h_sum.frames) == lay.n_frames
        s = torch.cuda.Stream(dev)
        engine.verify(desc, lay.n_frames, lay.seed, out, mism, stream=s)
        s.synchronize()
        assert int(mism.item()) == 0
    finally:
        engine.set_unmask_stream(None)


@pytest.mark.parametrize("zero_copy_max", [0, 1 << 30])
def test_protocol_pass_on_a_context_with_an_unmask_stream(engine, zero_copy_max):
    """The host protocol's multi-kernel pass (more than 256 connections) on a
    context whose decode ends on an unmask stream: its stream waits for the
    unmask, so the delivered payloads are the oracle's."""
    from oracle import ws_oracle as wo
    front, back, _ = _masked_streams(engine.device)
    rng = np.random.default_rng(31)
    streams = []
    for _ in range(300):
        s = b""
        for _ in range(int(rng.integers(1, 6))):
            L = int(rng.integers(0, 3000))
            s += wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), 2, True, 0, True,
                                 bytes(rng.integers(0, 256, 4, dtype=np.uint8)))
        streams.append(s)
    engine.set_unmask_stream(back)
    try:
        proto = gev_amd.Protocol(engine)
        proto.set_zero_copy_max(zero_copy_max)
        conns = [gev_amd.Connection() for _ in streams]
        rings = []
        for s in streams:
            r = gev_amd.RingBuffer(64)
            r.write(s)
            rings.append(r)
        n = proto.unpacket_batch(conns, rings)
        assert n == sum(len(wo.decode_stream(s).frames) for s in streams)
        for c, r, s in zip(conns, rings, streams):
            for fr in wo.decode_stream(s).frames:
                h, data = proto.unpacket(c, r)
                assert h is not None and h.length == fr.header.length
                assert data == fr.payload
    finally:
        engine.set_unmask_stream(None)
