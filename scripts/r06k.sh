# round 6: the resident decode service (k_decode_service, opt-in).  GPU
# tests first (the service's passes bit-exact against the oracle, its life
# cycle, the Protocol and live-server paths through it), then the live A/B.
# Predicted: C1 (100 connections, one loop) launch phase ~5.5 -> < 1 us a
# pass, wait still < 2 us (the pass overlaps the loop's socket reads),
# echoes/s +5 % (+-3 % run noise) -- about level with the CPU twin; WSS
# (8 loops): launch 12-20 -> < 1 us, echoes/s +5-15 % if the eight resident
# instances do not share hardware queues (a shared queue would show as
# signalled_share < 1 and waits of ~50 ms).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_service.py \
  tests/test_gpu_loopback.py::test_c1_loopback_resident_service > gpurun_out/r06k_pytest.log 2>&1 &&
TAG=r06k ROUNDS=3 timeout -k 10 400 bash scripts/lb_service_ab.sh
