# round 6: the resident service with only the workgroups that hold a slice
# joining a pass (r06k: all 32 counted in; C1's pass body 8.5 -> 12.5 us and
# its wait 0.2 -> 9 us, echoes/s -7 %).  Predicted: the body back to ~9 us,
# the wait ~3 us, C1 echoes/s level with the launched passes (+-3 %); the
# per-pass acquire fence's share read from the no-fence runs.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_service.py \
  tests/test_gpu_loopback.py::test_c1_loopback_resident_service > gpurun_out/r06l_pytest.log 2>&1 &&
TAG=r06l ROUNDS=3 SHAPES=C1 NOFENCE=1 timeout -k 10 300 bash scripts/lb_service_ab.sh
# (the no-fence runs used a measurement knob, GEVWS_SERVICE_FENCE=0, removed
# after this run: slower -- wait 27-31 us -- and unsafe for device-memory input)
