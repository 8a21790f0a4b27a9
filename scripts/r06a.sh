# round 6, first box: the two-shape one-launch decode + tagged hand-offs
# (parity at the limits, protocol + live-server tests), then the live sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
P=tests/test_gpu_parity.py
bash scripts/gpu.sh "test $P::test_one_launch_decode_at_its_limits $P::test_completion_flag_signals_one_launch_passes $P::test_golden_vectors $P::test_rfc6455_kats_on_device $P::test_alignment_and_length_sweep" 'test tests/test_gpu_protocol.py tests/test_gpu_loopback.py' && TAG=r06a PRIO_ALL=1 bash scripts/loopback_sweep.sh
