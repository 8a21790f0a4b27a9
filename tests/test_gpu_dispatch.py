"""GPU parity for control-frame dispatch: the device
HandlerWrap.OnMessage (plugins/websocket/wrap.go:38-90) with util.HandleClose /
HandlePing / HandlePong / CheckCloseFrameData (util/util.go:27-85), followed by
the device encoder -- the bytes a gev websocket server would send back --
against the oracle restatement, bit-exact, for each echo policy."""
import numpy as np
import pytest

import gev_amd
from oracle import ws_oracle as wo
from tests._helpers import gpu_decode, host_result, pack_streams

pytestmark = pytest.mark.gpu

UTF8_CASES = [b"", b"bye", "héllo wörld ✓ 日本".encode(), b"\xf0\x9f\x98\x80ok", b"\xff", b"\xc0\xaf",
              b"\xed\xa0\x80", b"\xe2\x82", b"\xf4\x90\x80\x80", b"\xf4\x8f\xbf\xbf", b"\xef\xbb\xbf",
              b"\xe0\x80\xaf", b"abc\x80", "x".encode() * 200, ("é" * 100).encode()]
CODES = [0, 1, 999, 1000, 1001, 1002, 1003, 1004, 1005, 1006, 1007, 1011, 1012, 1015, 1016, 2999, 3000, 4000,
         4999, 5000, 65535]


def _client_stream(rng, n):
    m = lambda: bytes(rng.integers(0, 256, 4, dtype=np.uint8))  # noqa: E731
    s = b""
    for _ in range(n):
        r = rng.random()
        if r < 0.35:
            L = int(rng.integers(0, 3000))
            s += wo.encode_frame(bytes(rng.integers(0, 256, L, dtype=np.uint8)), int(rng.choice([0, 1, 2, 3])),
                                 bool(rng.random() < .8), 0, True, m())
        elif r < 0.55:
            s += wo.encode_frame(bytes(rng.integers(0, 256, int(rng.integers(0, 126)), dtype=np.uint8)),
                                 int(rng.choice([9, 10])), True, 0, True, m())
        elif r < 0.9:
            kind = rng.random()
            if kind < 0.1:
                body = b""
            elif kind < 0.2:
                body = bytes([int(rng.integers(0, 256))])
            else:
                body = int(rng.choice(CODES)).to_bytes(2, "big") + UTF8_CASES[int(rng.integers(0, len(UTF8_CASES)))]
            s += wo.encode_frame(body, wo.OP_CLOSE, True, 0, True, m())
        else:
            s += wo.encode_frame(b"r" * int(rng.integers(0, 20)), int(rng.choice([0xB, 0xC, 0xF])), True, 0, True, m())
    return s


@pytest.mark.parametrize("policy,n_streams", [(gev_amd._abi.HANDLER_NONE, 30), (gev_amd._abi.HANDLER_ECHO_BINARY, 30),
                                               (gev_amd._abi.HANDLER_ECHO_TEXT, 30),
                                               (gev_amd._abi.HANDLER_ECHO_BINARY, 300)])
def test_dispatch_and_encode_replies(engine, policy, n_streams):
    """n_streams 300: ~9 000 frames, i.e. several dispatch / encode workgroups
    of 4 096 frames each and their carried reply / aux-slot / wire offsets."""
    rng = np.random.default_rng(50 + policy + n_streams)
    streams = [_client_stream(rng, int(rng.integers(1, 60))) for _ in range(n_streams)]
    arena, conns = pack_streams(streams)
    import torch
    dev = torch.device("cuda", engine.device)
    d_in = torch.zeros(len(arena) + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    d_in[: len(arena)] = torch.from_numpy(np.frombuffer(arena, np.uint8).copy()).to(dev)
    out = engine.decode(d_in, len(arena), torch.from_numpy(conns.copy()).to(dev), conns.shape[0],
                        aux_slots=8192)
    wire, reply_of, ds = engine.serve(out, policy)
    want, shut, reps = b"", 0, []
    k = 0
    for s in streams:
        for fr in wo.decode_stream(s).frames:
            r, sd = wo.on_message(fr.header, fr.payload, policy)
            shut += sd
            reps.append(-1 if r is None else k)
            if r is not None:
                want += r
                k += 1
    assert int(ds["errors"]) == shut
    assert int(ds["frames"]) == k
    assert list(reply_of) == reps
    got = wire.cpu().numpy().tobytes()
    assert len(got) == len(want)
    assert got == want


def test_close_reply_matrix(engine):
    """Every close code class x every UTF-8 case, one frame each."""
    import torch
    frames = []
    for code in CODES:
        for reason in UTF8_CASES:
            frames.append(wo.encode_frame(code.to_bytes(2, "big") + reason, wo.OP_CLOSE, True, 0, True, b"\x01\x02\x03\x04"))
    frames.append(wo.encode_frame(b"", wo.OP_CLOSE, True, 0, True, b"\x01\x02\x03\x04"))
    frames.append(wo.encode_frame(b"\x03", wo.OP_CLOSE, True, 0, False))
    s = b"".join(frames) + b"\x82\x7f\x00\x00\x00"
    dev = torch.device("cuda", engine.device)
    d_in = torch.zeros(len(s) + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    d_in[: len(s)] = torch.from_numpy(np.frombuffer(s, np.uint8).copy()).to(dev)
    out = engine.decode(d_in, len(s), torch.tensor([[0, len(s)]], dtype=torch.int64, device=dev), 1,
                        aux_slots=len(frames))
    wire, _, ds = engine.serve(out, gev_amd._abi.HANDLER_NONE)
    want = b"".join(wo.on_message(fr.header, fr.payload, 0)[0] for fr in wo.decode_stream(s).frames)
    assert wire.cpu().numpy().tobytes() == want
    assert int(ds["errors"]) == len(frames)


@pytest.mark.parametrize("policy,n_streams", [(gev_amd._abi.HANDLER_ECHO_TEXT, 12), (gev_amd._abi.HANDLER_NONE, 12),
                                               (gev_amd._abi.HANDLER_ECHO_BINARY, 300)])
def test_handle_decoded_one_launch_matches_two_steps(engine, policy, n_streams):
    """gevws_handle_decoded_async (a live pass's handler step behind its
    decode, no host round trip): with <= 1 024 frames it is ONE launch
    (k_handle_small), else the dispatch + encode chain; either way the wire
    bytes, reply_of and both summaries equal the oracle's replies and the
    two-step path's, also with a frame bound above the decoded count."""
    import torch
    rng = np.random.default_rng(77 + policy + n_streams)
    streams = [_client_stream(rng, int(rng.integers(1, 60))) for _ in range(n_streams)]
    arena, conns = pack_streams(streams)
    dev = torch.device("cuda", engine.device)
    d_in = torch.zeros(len(arena) + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    d_in[: len(arena)] = torch.from_numpy(np.frombuffer(arena, np.uint8).copy()).to(dev)
    want, shut, reps, nrep = b"", 0, [], 0
    for s in streams:
        for fr in wo.decode_stream(s).frames:
            r, sd = wo.on_message(fr.header, fr.payload, policy)
            shut += sd
            reps.append(-1 if r is None else nrep)
            if r is not None:
                want += r
                nrep += 1
    nf = len(reps)
    aux = max(nf, 1)
    for bound in sorted({nf, nf + 37, nf + 1100}):  # (a bound below nf handles only its first frames)
        out = engine.decode(d_in, len(arena), torch.from_numpy(conns.copy()).to(dev), conns.shape[0],
                            aux_slots=aux)
        wire, reply_of, ds, es = engine.handle_decoded(out, policy, bound, aux, len(want) + 64)
        assert int(ds["status"]) == 0 and int(es["status"]) == 0, bound
        assert int(ds["frames"]) == nrep and int(ds["errors"]) == shut, bound
        assert int(es["frames"]) == nrep and int(es["payload_bytes"]) == len(want), bound
        assert list(reply_of) == reps, bound
        assert wire.cpu().numpy().tobytes() == want, bound
