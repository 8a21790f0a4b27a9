# round 6, final tree: the GPU test files not re-run since the DPP-scan and
# record-pass changes (r06ab / r06ad ran the decode, encode, dispatch, split,
# property, protocol, service and direct files): loopback, bench, comm; then
# smoke().  Together with r06ab / r06ad this covers every GPU test file on
# the final kernels without a third full-suite run.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_loopback.py \
  tests/test_gpu_bench.py tests/test_gpu_comm.py > gpurun_out/r06ah_pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/run_smoke.py > gpurun_out/r06ah_smoke.log 2>&1
