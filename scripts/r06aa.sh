# round 6: the one-launch decode's block scan on DPP wave scans (32-bit sums)
# instead of the 64-bit shuffle scan, whose ds_bpermute round trips took 2.5
# us of the 8.6 us kernel (r06z, GEVWS_PHASE_TICKS).  Predicted: scan 2.5 ->
# ~0.3 us, kernel 8.6 -> ~6.4 us, post -> signal -2 us on every placement.
# Parity first: the one-launch tests (limits, both shapes, live passes, the
# hypothesis properties incl. flagged passes), service, direct, protocol.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_properties.py tests/test_gpu_service.py tests/test_gpu_direct.py tests/test_gpu_protocol.py \
  > gpurun_out/r06aa_pytest.log 2>&1 &&
GEVWS_PHASE_TICKS=1 timeout -k 10 300 python -u tools/live_pass_probe.py --reps 300 > gpurun_out/r06aa_live_pass_phases.jsonl 2> gpurun_out/r06aa.err
