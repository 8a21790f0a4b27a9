"""TestWebSocketServer_CloseConnection (example/websocket/wsserver_test.go:135-178)
on the CPU: the loopback server's connection accounting (OnConnect at accept,
OnClose when the loop closes the connection, connection.go:288-303) with the
CPU-decode twin (tools/ws_loopback_cpu), 8 loops, 10 clients, 5 closed by a
bare TCP close.  The device-decode server runs the same check, close frames
included, in tests/test_gpu_loopback.py."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_close_connection_counts_cpu_twin():
    path = os.path.join(ROOT, "tools", "ws_loopback_cpu")
    if not os.path.exists(path):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tools")], check=True, capture_output=True, timeout=300)
    r = subprocess.run([path, "--mode", "close", "--conns", "10", "--to-close", "5", "--loops", "8",
                        "--close-frame", "0"], capture_output=True, text=True, timeout=60)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, (r.stdout[-1500:], r.stderr[-1500:])
    d = json.loads(lines[0])
    assert d["upgraded"] == 10 and d["errors"] == 0
    assert (d["live_after_connect"], d["live_after_close"], d["live_at_end"]) == (10, 5, 0)
