# round 6, final tree (decode body in gevws_small.hpp): the GPU test files
# r06ak did not run -- properties, split, encode, bench, comm -- and smoke,
# so every GPU test file has run on the final build (with r06ak).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_properties.py \
  tests/test_gpu_split.py tests/test_gpu_encode.py tests/test_gpu_bench.py tests/test_gpu_comm.py \
  > gpurun_out/r06al_pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/run_smoke.py > gpurun_out/r06al_smoke.log 2>&1
