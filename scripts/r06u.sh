# round 6: r06t (final tree, another box) had the wsserver shape 10-20 %
# below the round's service commit (ab_base/): 267-298 k against 330-339 k,
# its decode kernel 9.8-10.6 against 9.4-9.5 us -- the decode's lazy
# last-call event behind a recorded handler step (r06n had measured it level
# or better on its box).  This build keeps the lazy record only for a
# one-launch decode that follows another (C1's rhythm); a decode after a
# handler step records as before.  Predicted: wsserver level with ab_base
# (+-5 %), C1's launch phase still ~3.6 us.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_protocol.py \
  tests/test_gpu_parity.py::test_own_stream_live_pass_then_other_stream_is_ordered \
  tests/test_gpu_parity.py::test_one_context_two_streams_is_ordered tests/test_gpu_dispatch.py > gpurun_out/r06u_pytest.log 2>&1 &&
TAG=r06u ROUNDS=3 SHAPES="WSS C1" timeout -k 10 500 bash scripts/lb_ab.sh
