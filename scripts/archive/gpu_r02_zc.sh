#!/bin/bash
# Host-ingress protocol tests, then the C1 loopback with zero-copy small passes
# (default) against copy-in/copy-out passes (GEVWS_LB_ZERO_COPY_MAX=0) and the
# CPU-decode server, interleaved.
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_loopback.py -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $OUT/zc_tests.log 2>&1
rc=$?; tail -3 $OUT/zc_tests.log; [ $rc -eq 0 ] || exit $rc
export GEV_LOG_LEVEL=FATAL
run() { local name=$1; shift; timeout -k 10 60 "$@" > $OUT/$name.log 2> $OUT/$name.err || { tail -3 $OUT/$name.err; exit 1; }; cat $OUT/$name.log; }
for rnd in 1 2; do
  run zc_dev_$rnd gev_amd/ws_loopback --conns 100 --loops 1 --msg 128 --seconds 3 --client-threads 2
  GEVWS_LB_ZERO_COPY_MAX=0 run cp_dev_$rnd gev_amd/ws_loopback --conns 100 --loops 1 --msg 128 --seconds 3 --client-threads 2
  run cpu_$rnd tools/ws_loopback_cpu --conns 100 --loops 1 --msg 128 --seconds 3 --client-threads 2
done
run zc_dev4 gev_amd/ws_loopback --conns 4000 --loops 4 --msg 128 --seconds 3 --client-threads 8
GEVWS_LB_ZERO_COPY_MAX=0 run cp_dev4 gev_amd/ws_loopback --conns 4000 --loops 4 --msg 128 --seconds 3 --client-threads 8
run cpu4 tools/ws_loopback_cpu --conns 4000 --loops 4 --msg 128 --seconds 3 --client-threads 8
