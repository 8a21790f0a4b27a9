# round 6: C1 launched vs direct dispatch again, now that the one-launch
# kernel is 6.4 us (DPP scans; r06q/r06r measured direct level with a 8.6 us
# kernel: launch 3.6 -> 1.0 us but wait 0.3 -> 2.8 us).  Predicted: direct's
# wait back under 1 us, its launch + wait ~2.5 us under the launched pass's,
# echoes/s +1-3 % (inside C1's run spread, so read from the timeline).
# (The direct tests first: its kernarg slots now track use explicitly.)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_direct.py \
  tests/test_gpu_loopback.py::test_c1_loopback_direct_dispatch > gpurun_out/r06ae_pytest.log 2>&1 &&
TAG=r06ae ROUNDS=3 SHAPES=C1 NO_SVC=1 DIRECT=1 timeout -k 10 400 bash scripts/lb_service_ab.sh
