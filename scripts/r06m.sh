# round 6: one-launch calls on the context's own stream leave their
# last-call event unrecorded until something needs it (mark_last_lazy): a
# live pass saves one hipEventRecord (two with the handler step chained).
# Predicted: C1 launch phase 5.5 -> ~4.5 us a pass, echoes/s +1-2 % (run
# noise +-3 %); wsserver launch 12-20 -> ~10-17 us.  Ordering tests first
# (streams, protocol, service, loopback), then this build against the
# previous commit's (ab_base/) and the CPU twin, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_protocol.py \
  tests/test_gpu_service.py tests/test_gpu_loopback.py tests/test_gpu_dispatch.py \
  tests/test_gpu_parity.py::test_own_stream_live_pass_then_other_stream_is_ordered tests/test_gpu_parity.py::test_one_context_two_streams_is_ordered > gpurun_out/r06m_pytest.log 2>&1 &&
TAG=r06m ROUNDS=3 SHAPES="C1 WSS" timeout -k 10 400 bash scripts/lb_ab.sh
