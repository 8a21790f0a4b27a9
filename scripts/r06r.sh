# round 6: r06q's direct dispatch cut C1's launch phase 3.4-3.7 -> 1.0-1.2 us
# but its wait rose 0.2-0.8 -> 2.5-3.1 us and the kernel's own time 8.6 ->
# 9.4 us: net level with launched passes.  This run puts the packets' acquire
# / release fences at agent scope (HIP's own choice for kernels whose inputs
# the host did not just write is unknown here).  Predicted: if the system-
# scope fences cost the ~1.5 us of start latency, the wait back under 1 us and
# C1 echoes/s +3 % over the launched passes; else no change (then dropped).
# The direct tests run first with agent scope (device-memory inputs reused
# across passes: a stale line would show as a mismatch).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
GEVWS_DIRECT_SCOPE=agent timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_direct.py > gpurun_out/r06r_pytest.log 2>&1 &&
TAG=r06r ROUNDS=3 SHAPES=C1 NO_SVC=1 DIRECT=1 DIRECT_AGENT=1 timeout -k 10 300 bash scripts/lb_service_ab.sh
# (GEVWS_DIRECT_SCOPE, the measurement knob this run used, was removed after
# it: agent scope measured within run noise of system scope)
