# round 6: every block scan on DPP wave scans (block_excl_scan, 64-bit: the
# walk's block counts, the partials scan, encode, dispatch and the one-
# workgroup handler step; block_excl_scan32 in the one-launch decode, r06aa).
# The change reaches every decode and encode kernel, so their test files run
# (not the whole suite: no loopback / bench / comm files).  Then C3 / C4 /
# C2 bench lines (predicted: within +-1 % -- the scans are a sliver of those
# kernels), the live-pass probe (handler-free, as r06aa) and the live shapes
# against ab_base (predicted: wsserver's handler step -2-3 us a pass, echoes
# within noise).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_properties.py tests/test_gpu_encode.py tests/test_gpu_dispatch.py tests/test_gpu_split.py \
  tests/test_gpu_protocol.py tests/test_gpu_service.py tests/test_gpu_direct.py > gpurun_out/r06ab_pytest.log 2>&1 &&
JSONL=r06ab_bench bash scripts/gpu.sh 'bench r06ab_c3 --config c3 --steps 5' 'bench r06ab_c4 --config c4 --steps 5' \
  'bench r06ab_c2 --config c2' 'bench r06ab_c5 --config c5' &&
GEVWS_PHASE_TICKS=1 timeout -k 10 300 python -u tools/live_pass_probe.py --reps 300 > gpurun_out/r06ab_live_pass_phases.jsonl 2> gpurun_out/r06ab.err &&
TAG=r06ab ROUNDS=3 SHAPES="WSS C1" timeout -k 10 500 bash scripts/lb_ab.sh
