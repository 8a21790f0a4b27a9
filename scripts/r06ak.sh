# round 6: after taking the fused decode + handler launch out again (r06aj:
# wsserver -45 %), the tree keeps only the decode body's move into
# gevws_small.hpp.  The one-launch / protocol / dispatch / loopback tests,
# then wsserver and C1 against ab_base: predicted back at r06ab's level
# (wsserver within the shape's spread of the base).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dispatch.py \
  tests/test_gpu_protocol.py tests/test_gpu_parity.py tests/test_gpu_service.py tests/test_gpu_direct.py \
  tests/test_gpu_loopback.py > gpurun_out/r06ak_pytest.log 2>&1 &&
TAG=r06ak ROUNDS=2 SHAPES="WSS C1" timeout -k 10 400 bash scripts/lb_ab.sh
