# round 6: direct dispatch claims its AQL packet and kernarg slots only after
# both waits succeed (a failed wait no longer leaves a claimed, empty packet
# slot); the live-pass test helpers moved into tests/_helpers.py.  The
# direct, service and ordering tests again.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_direct.py \
  tests/test_gpu_service.py tests/test_gpu_loopback.py::test_c1_loopback_direct_dispatch \
  tests/test_gpu_loopback.py::test_c1_loopback_resident_service \
  tests/test_gpu_parity.py::test_own_stream_live_pass_then_other_stream_is_ordered > gpurun_out/r06v_pytest.log 2>&1
