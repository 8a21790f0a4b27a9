# round 6: direct dispatch (gev_amd/csrc/gevws_direct.cpp, opt-in): a live
# pass written as one AQL packet into the context's own HSA queue.  Tests
# first (a wrong packet would fault: each step under its own limit), then
# the live A/B.  Predicted: C1 launch phase 3.6 -> < 1 us a pass, the wait
# unchanged (< 1 us: the pass still overlaps the socket reads; the kernel
# reads its 120-byte kernarg from host memory, ~1 us more start latency),
# echoes/s +3-5 %; the wsserver shape unchanged (its passes chain the
# handler step, so they still launch).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest -x -v --timeout 60 --timeout-method thread \
  tests/test_gpu_direct.py::test_direct_synchronize_and_off > gpurun_out/r06q_pytest.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_direct.py \
  tests/test_gpu_loopback.py::test_c1_loopback_direct_dispatch tests/test_gpu_service.py >> gpurun_out/r06q_pytest.log 2>&1 &&
TAG=r06q ROUNDS=3 SHAPES=C1 DIRECT=1 timeout -k 10 300 bash scripts/lb_service_ab.sh
