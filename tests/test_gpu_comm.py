"""Multi-GPU at the C ABI for one process driving several
GPUs: gevws_comm (ncclCommInitAll over the process's devices) and the decode
path's one collective, the all-reduce(sum) of each device's decoded {frames,
payload bytes, errors}.  On a one-GPU box the communicator has one rank (the
reduce is then the identity -- still the RCCL path end to end); the N > 1 case
runs where the box has the devices.  The one-process-per-GPU form (bench.py over
torch.distributed) is covered by tests/test_dist_gloo.py and test_gpu_bench.py."""
import numpy as np
import pytest

import gev_amd
from oracle import ref
from tests._helpers import gpu_decode, pack_streams, random_stream

pytestmark = pytest.mark.gpu


def _batch(seed, n=40):
    rng = np.random.default_rng(seed)
    return pack_streams([random_stream(rng, int(rng.integers(0, 30))) for _ in range(n)])


def test_counts_allreduce_one_device(engine):
    comm = gev_amd.Comm([engine.device])
    assert comm.size() == 1
    arena, conns = _batch(41)
    out = gpu_decode(engine, arena, conns)
    want = ref.decode_batch(np.frombuffer(arena, np.uint8).copy(), conns[:, 0], conns[:, 1])
    tot = comm.allreduce_counts([engine], [out])
    assert tot == (want["frames"].shape[0], int(want["frames"]["length"].sum()),
                   int((want["conn_status"] < 0).sum()))
    assert tuple(int(x) for x in out.counts.cpu()) == tot


def test_counts_allreduce_after_unsynchronised_decode(engine):
    """decode_async on torch's stream, then the reduce at once, with no
    synchronisation between them: the reduce must wait for the decode's summary
    (ADVICE r3).  A 4 GiB-payload C3-shaped batch keeps the decode running
    long after the host returns from the launch."""
    import torch
    from gev_amd import workloads as w
    lay = w.config_c3(seed=11, n_conns=1024, n_frames=1 << 16)
    dev = torch.device("cuda", engine.device)
    arena = torch.empty(lay.arena_bytes + gev_amd.IN_PAD, dtype=torch.uint8, device=dev)
    arena[lay.arena_bytes:] = 0
    desc = torch.from_numpy(lay.desc.view(np.uint8).copy()).to(dev)
    conns = torch.from_numpy(lay.conns.copy()).to(dev)
    engine.synth(arena, desc, lay.n_frames, lay.seed)
    out = engine.alloc_batch(lay.n_conns, lay.n_frames, lay.payload_padded)
    comm = gev_amd.Comm([engine.device])
    side = torch.cuda.Stream(dev)  # neither torch's current stream nor the context's own
    for _ in range(3):
        out.summary.zero_()
        side.wait_stream(torch.cuda.current_stream(dev))
        engine.decode_async(arena, lay.arena_bytes, conns, lay.n_conns, out, lay.n_frames, lay.payload_padded,
                            stream=side)
        tot = comm.allreduce_counts([engine], [out])
        assert tot == (lay.n_frames, lay.payload_len, 0)


def test_comm_rejects_bad_arguments(engine):
    with pytest.raises(RuntimeError):
        gev_amd.Comm([gev_amd.device_count() + 3])
    comm = gev_amd.Comm([engine.device])
    with pytest.raises(ValueError):
        comm.allreduce_counts([engine, engine], [None, None])


def test_counts_allreduce_every_device():
    """Each visible GPU decodes its own batch; every device ends up with the
    sum (skipped on a one-GPU box)."""
    n = gev_amd.device_count()
    if n < 2:
        pytest.skip("one GPU: the N > 1 reduce needs more devices")
    engines = [gev_amd.Engine(d) for d in range(n)]
    comm = gev_amd.Comm(list(range(n)))
    outs, want = [], [0, 0, 0]
    for d, e in enumerate(engines):
        arena, conns = _batch(50 + d)
        outs.append(gpu_decode(e, arena, conns))
        w = ref.decode_batch(np.frombuffer(arena, np.uint8).copy(), conns[:, 0], conns[:, 1])
        want[0] += w["frames"].shape[0]
        want[1] += int(w["frames"]["length"].sum())
        want[2] += int((w["conn_status"] < 0).sum())
    tot = comm.allreduce_counts(engines, outs)
    assert list(tot) == want
    for o in outs:
        assert [int(x) for x in o.counts.cpu()] == want


def test_two_devices_comm_and_loopback_server():
    """The in-process multi-GPU path on the first box with two GPUs (VERDICT r4
    item 1): a two-device communicator reducing two devices' decodes, then the
    live loopback server with its loops on two devices round-robin
    (load_balance.go:7-14), every echo checked by its client.  Skipped only
    when fewer than two GPUs are visible."""
    n = gev_amd.device_count()
    if n < 2:
        pytest.skip(f"{n} GPU(s) visible: the two-device path needs 2")
    engines = [gev_amd.Engine(d) for d in (0, 1)]
    comm = gev_amd.Comm([0, 1])
    assert comm.size() == 2
    outs, want = [], [0, 0, 0]
    for d, e in enumerate(engines):
        arena, conns = _batch(70 + d, n=60)
        out = gpu_decode(e, arena, conns)
        w = ref.decode_batch(np.frombuffer(arena, np.uint8).copy(), conns[:, 0], conns[:, 1])
        assert out.frames_host().tobytes() == w["frames"].tobytes()  # each device decodes bit-exact
        outs.append(out)
        want[0] += w["frames"].shape[0]
        want[1] += int(w["frames"]["length"].sum())
        want[2] += int((w["conn_status"] < 0).sum())
    assert list(comm.allreduce_counts(engines, outs)) == want
    for o in outs:
        assert [int(x) for x in o.counts.cpu()] == want
    from tests.test_gpu_loopback import _run
    d = _run("gev_amd/ws_loopback", conns=64, seconds=1.0, loops=4, threads=2,
             extra=("--mode", "wsserver", "--devices", "2"))
    assert d["devices"] == 2 and d["client_checked_echoes"] > 0 and d["errors"] == 0
