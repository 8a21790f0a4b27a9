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
