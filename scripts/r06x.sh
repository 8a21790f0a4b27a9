# round 6: direct dispatch and the resident service switched on one context
# (re-run after the direct queue got its error callback)
# (tests/test_gpu_direct.py::test_direct_and_service_on_one_context), with
# the ABI-3 build; the direct and service tests again.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_direct.py \
  tests/test_gpu_service.py > gpurun_out/r06x_pytest.log 2>&1
