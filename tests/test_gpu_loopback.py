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


def _run(binary, conns=100, seconds=2.0, msg=128, loops=1, threads=2, env=None, extra=()):
    path = os.path.join(ROOT, binary)
    assert os.path.exists(path), f"{binary} not built (python -c 'import __graft_entry__ as g; g.build()')"
    r = subprocess.run([path, "--conns", str(conns), "--seconds", str(seconds), "--msg", str(msg), "--loops",
                        str(loops), "--client-threads", str(threads), *extra], capture_output=True, text=True,
                       timeout=120, env={**os.environ, **(env or {})})
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


@pytest.mark.parametrize("msg,ways", [(128, 2), (128, 4), (65536, 3)])
def test_c1_loopback_split_passes(msg, ways):
    """GEVWS_LB_SPLIT=2: an iteration makes W device passes on W decoders
    (connections dealt to them at accept), group g's in flight while the
    later groups' sockets are read; every echo checked byte for byte,
    including 64 KiB frames carried across reads."""
    _run("gev_amd/ws_loopback", conns=100 if msg == 128 else 16, seconds=1.5, msg=msg,
         env={"GEVWS_LB_SPLIT": "2", "GEVWS_LB_WAYS": str(ways)})


def test_wsserver_mirror_split_passes_with_control_frames(tmp_path):
    """The wsserver mirror with split passes: control replies and closes still
    answered by each half's device handler (the oracle's replies)."""
    from oracle import ws_oracle as wo
    tr = tmp_path / "transcript.txt"
    d = _run("gev_amd/ws_loopback", conns=100, seconds=1.5, loops=2, threads=4,
             env={"GEVWS_LB_SPLIT": "2"},
             extra=("--mode", "wsserver", "--ctrl", "0.3", "--close-end", "1", "--transcript", str(tr)))
    assert d["closes_answered"] == 100
    for sent_hex, reply_hex in (ln.split() for ln in tr.read_text().splitlines() if ln.strip()):
        fr = wo.decode_stream(bytes.fromhex(sent_hex)).frames
        want, _ = wo.on_message(fr[0].header, fr[0].payload, wo.HANDLER_ECHO_TEXT)
        assert bytes.fromhex(reply_hex) == want


# ---------------------------------------------------------------- wsserver_test.go on the live server
def test_wsserver_test_mirror_8_loops_100_clients():
    """example/websocket/wsserver_test.go:73-133, the reference's own hot-path
    test: 8 loops, 100 clients for 2 s, each sending masked text frames of
    random 1..3072 bytes and reading the echo back in full (bytes.Equal); the
    server answers (MessageText, data) by return value or by c.Send(PackData)
    at random (:47-63).  Here the answer of every frame is computed on the
    device (the protocol's handler step: HandlerWrap.OnMessage + FrameToBytes)
    and both routes are taken; zero mismatches."""
    d = _run("gev_amd/ws_loopback", conns=100, seconds=2.0, loops=8, threads=4, extra=("--mode", "wsserver"))
    assert d["mode"] == "wsserver" and d["decoder"] == "device"
    assert d["client_checked_echoes"] > 1000
    assert d["async_sends"] > 0  # both reply routes taken


def test_wsserver_mirror_cpu_twin_beside():
    """The same mirror on the CPU-decode twin (host-framed text echo): the
    baseline server passes the reference test's checks too."""
    d = _run("tools/ws_loopback_cpu", conns=100, seconds=2.0, loops=8, threads=4, extra=("--mode", "wsserver"))
    assert d["client_checked_echoes"] > 1000


def test_wsserver_control_frames_match_oracle(tmp_path):
    """Control frames on the live server, answered by the device dispatch
    inside the loop: clients put a masked ping (or pong) before 30 % of their
    messages and end with a close frame (valid / reserved / unknown /
    application codes, UTF-8 and invalid reasons, empty bodies).  Every reply
    the clients received -- pong for ping, the reference's ping for pong
    (util.go:54-56), util.HandleClose's close reply -- is compared byte for
    byte with oracle/ws_oracle.on_message for the frame they sent, and every
    close is followed by the server's ShutdownWrite (the client sees EOF)."""
    from oracle import ws_oracle as wo
    tr = tmp_path / "transcript.txt"
    d = _run("gev_amd/ws_loopback", conns=100, seconds=1.5, loops=8, threads=4,
             extra=("--mode", "wsserver", "--ctrl", "0.3", "--close-end", "1", "--transcript", str(tr)))
    assert d["closes_answered"] == 100
    pairs = [ln.split() for ln in tr.read_text().splitlines() if ln.strip()]
    assert len(pairs) == d["transcript_pairs"] and len(pairs) >= 100 + 50
    kinds = set()
    for sent_hex, reply_hex in pairs:
        sent = bytes.fromhex(sent_hex)
        fr = wo.decode_stream(sent).frames
        assert len(fr) == 1
        want, shut = wo.on_message(fr[0].header, fr[0].payload, wo.HANDLER_ECHO_TEXT)
        assert bytes.fromhex(reply_hex) == want, (fr[0].header, fr[0].payload)
        assert shut == (fr[0].header.opcode == wo.OP_CLOSE)
        kinds.add(fr[0].header.opcode)
    assert kinds == {wo.OP_PING, wo.OP_PONG, wo.OP_CLOSE}


def test_wsserver_loops_placed_on_devices_round_robin():
    """--devices N places loop l on device l % N (one context + protocol per
    loop); on a one-GPU box N = the visible devices (1), the mapping still goes
    through the flag."""
    import gev_amd
    n = max(1, gev_amd.device_count())
    d = _run("gev_amd/ws_loopback", conns=64, seconds=1.0, loops=4, threads=2,
             extra=("--mode", "wsserver", "--devices", str(n)))
    assert d["devices"] == n and d["client_checked_echoes"] > 0


# ---------------------------------------------------------------- wsserver_test.go:135-178
def _run_close(binary, close_frame):
    path = os.path.join(ROOT, binary)
    assert os.path.exists(path), f"{binary} not built"
    r = subprocess.run([path, "--mode", "close", "--conns", "10", "--to-close", "5", "--loops", "8",
                        "--close-frame", str(close_frame)], capture_output=True, text=True, timeout=60)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (r.returncode, r.stdout[-1500:], r.stderr[-1500:])
    d = json.loads(lines[0])
    print(binary, json.dumps(d))
    assert r.returncode == 0, d
    return d


@pytest.mark.parametrize("close_frame", [1, 0])
def test_wsserver_close_connection_mirror(close_frame):
    """TestWebSocketServer_CloseConnection (wsserver_test.go:135-178) on the
    device-decode server: 8 loops, 10 clients dial and upgrade (OnConnect count
    10), 5 close -- with a close frame first, as x/net/websocket's Conn.Close
    (answered on the device: close reply + ShutdownWrite), or a bare TCP close
    -- and after the drain the OnConnect - OnClose count is 5, then 0."""
    d = _run_close("gev_amd/ws_loopback", close_frame)
    assert d["decoder"] == "device"
    assert (d["live_after_connect"], d["live_after_close"], d["live_at_end"]) == (10, 5, 0)
    if close_frame:
        assert d["closes_answered"] == 5


def test_c1_loopback_resident_service():
    """GEVWS_LB_SERVICE=1: the live server's zero-copy passes are posted to the
    context's resident decode service (no launch call); every echo is still
    checked byte for byte, and the passes really went there."""
    d = _run("gev_amd/ws_loopback", conns=100, seconds=1.5, env={"GEVWS_LB_SERVICE": "1"})
    tl = d["pass_timeline_us"]
    assert tl["service_share"] > 0.9 and tl["signalled_share"] > 0.9, tl


def test_c1_loopback_direct_dispatch():
    """GEVWS_LB_DIRECT=1: the live server's zero-copy passes are written into
    each context's own AQL queue; every echo still checked byte for byte."""
    d = _run("gev_amd/ws_loopback", conns=100, seconds=1.5, env={"GEVWS_LB_DIRECT": "1"})
    tl = d["pass_timeline_us"]
    assert tl["direct_share"] > 0.9 and tl["signalled_share"] > 0.9, tl
