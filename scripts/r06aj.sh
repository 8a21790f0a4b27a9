# round 6: a live pass's decode and handler step in ONE launch
# (gevws_decode_handle_async / k_decode_handle_small: the decoding workgroup
# goes on to dispatch and encode); the Protocol's zero-copy passes with a
# handler use it.  Under the wsserver shape the gap before the separately
# dispatched handler kernel was ~38 us of a ~73 us wait (r06ai).  Parity
# first: the new entry's test, the dispatch / handler / protocol / loopback
# files (the decode body moved into gevws_small.hpp: the one-launch and
# property tests too).  Predicted: wsserver's gpu_gap 38 -> < 1 us, its wait
# 73 -> ~35 us, its launch phase 15 -> ~9 us; echoes/s within the shape's
# spread (its clients bound it: the CPU twin is level).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dispatch.py \
  tests/test_gpu_protocol.py tests/test_gpu_parity.py tests/test_gpu_properties.py tests/test_gpu_service.py \
  tests/test_gpu_direct.py tests/test_gpu_loopback.py > gpurun_out/r06aj_pytest.log 2>&1 &&
TAG=r06aj ROUNDS=3 SHAPES="WSS C1" timeout -k 10 500 bash scripts/lb_ab.sh
# (measured: wsserver 198 / 174 k against the base's 345 / 336 k -- launch
# 24-31 us, decode part 10.6-11.5 us: 45 % slower, so the fused pass was
# taken out again; the decode body stays in gevws_small.hpp)
