"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only):
the ring buffer of the C++ host mirror fuzzed against a std::deque model, and
the C oracle's decode on random hostile byte streams, and the HTTP upgrade
(gev_amd/csrc/handshake.cpp) on mutated requests (race /
sanitizer coverage is host-side; GPU ASan is not available on this pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all", "-g", "-O1"]


def _run(cmd, **kw):
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300, **kw)


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_ring_buffer_fuzz_asan_ubsan(tmp_path):
    exe = tmp_path / "ring_fuzz"
    r = _run(["g++", "-std=c++17", *SAN, os.path.join(ROOT, "tests", "cpp", "ring_fuzz.cpp"), "-o", str(exe)])
    assert r.returncode == 0, r.stderr
    for seed in ("1", "2", "3"):
        r = _run([str(exe), seed], env={**os.environ, "ASAN_OPTIONS": "detect_leaks=1"})
        assert r.returncode == 0 and "ring_fuzz ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no host C compiler")
def test_oracle_decode_fuzz_asan_ubsan(tmp_path):
    exe = tmp_path / "oracle_fuzz"
    r = _run(["gcc", "-std=c11", "-D_POSIX_C_SOURCE=199309L", *SAN,
              os.path.join(ROOT, "tests", "cpp", "oracle_fuzz.c"), os.path.join(ROOT, "oracle", "ws_ref.c"),
              "-lpthread", "-o", str(exe)])
    assert r.returncode == 0, r.stderr
    r = _run([str(exe)], env={**os.environ, "ASAN_OPTIONS": "detect_leaks=1"})
    assert r.returncode == 0 and "oracle_fuzz ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_handshake_fuzz_asan_ubsan(tmp_path):
    exe = tmp_path / "handshake_fuzz"
    r = _run(["g++", "-std=c++17", *SAN, "-I", os.path.join(ROOT, "include"),
              os.path.join(ROOT, "tests", "cpp", "handshake_fuzz.cpp"),
              os.path.join(ROOT, "gev_amd", "csrc", "handshake.cpp"), "-o", str(exe)])
    assert r.returncode == 0, r.stderr
    r = _run([str(exe)], env={**os.environ, "ASAN_OPTIONS": "detect_leaks=1"})
    assert r.returncode == 0 and "handshake_fuzz ok" in r.stdout, r.stdout + r.stderr
