"""C1 (BASELINE config 1, plumbing): the live loopback echo server over the C
ABI, as benchmarks/bench-websocket-pingpong.sh:25-28 drives gev's websocket
server (benchmarks/websocket/server.go:22-29) but with 1 work loop and 128-byte
masked text frames -- real sockets, ring buffers fed by read(2), one device
pass per loop iteration, UnPacket, binary echo.  The in-process clients check
every echoed byte; any mismatch, lost connection or handshake failure fails
the test.  The CPU-decode build of the same server (tools/ws_loopback_cpu,
oracle/ws_ref.c's per-frame pipeline) runs beside it as the baseline and must
echo correctly too."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(binary, conns=100, seconds=2.0, msg=128, loops=1, threads=2, env=None):
    path = os.path.join(ROOT, binary)
    assert os.path.exists(path), f"{binary} not built (python -c 'import __graft_entry__ as g; g.build()')"
    r = subprocess.run([path, "--conns", str(conns), "--seconds", str(seconds), "--msg", str(msg), "--loops",
                        str(loops), "--client-threads", str(threads)], capture_output=True, text=True, timeout=120,
                       env={**os.environ, **(env or {})})
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.returncode, r.stdout[-1500:], r.stderr[-1500:])
    d = json.loads(lines[0])
    print(binary, json.dumps(d))
    assert d["errors"] == 0 and d["upgraded"] == conns
    assert d["echoes_per_s"] > 0 and d["client_checked_echoes"] > 0
    return d


def test_c1_loopback_device_decode():
    d = _run("gev_amd/ws_loopback")
    assert d["decoder"] == "device" and d["decode_passes_per_s"] > 0


def test_c1_loopback_cpu_baseline_beside():
    dev = _run("gev_amd/ws_loopback")
    cpu = _run("tools/ws_loopback_cpu")
    assert cpu["decoder"].startswith("cpu")
    print(json.dumps({"c1_echoes_per_s": {"device": dev["echoes_per_s"], "cpu": cpu["echoes_per_s"]}}))


def test_c1_loopback_large_frames_span_reads():
    """64 KiB messages: every frame spans several read(2)s, so partial frames
    wait in the ring for the next pass (the completeness carry)."""
    d = _run("gev_amd/ws_loopback", conns=16, seconds=1.5, msg=65536)
    assert d["client_checked_echoes"] > 0


@pytest.mark.parametrize("msg", [128, 65536])
def test_c1_loopback_pipelined_loop(msg):
    """GEVWS_LB_PIPELINE=1: the device pass of one loop iteration in flight
    (gevws_protocol_unpacket_batch_begin) while the next reads its sockets,
    ended (_end) before its frames are echoed and before any connection it
    holds is closed; every echo still checked byte for byte."""
    _run("gev_amd/ws_loopback", conns=100 if msg == 128 else 16, seconds=1.5, msg=msg,
         env={"GEVWS_LB_PIPELINE": "1"})
