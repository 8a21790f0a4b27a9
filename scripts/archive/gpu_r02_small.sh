#!/bin/bash
# Whole GPU suite, then the C1 loopback: device decode (one-launch small
# batches, zero-copy) vs multi-kernel small batches vs the CPU decode.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
export GEV_LOG_LEVEL=FATAL
run() { local name=$1; shift; timeout -k 10 60 "$@" > $OUT/$name.log 2> $OUT/$name.err || { tail -3 $OUT/$name.err; exit 1; }; cat $OUT/$name.log; }
for rnd in 1 2; do
  run sm_dev_$rnd gev_amd/ws_loopback --conns 100 --loops 1 --msg 128 --seconds 3 --client-threads 2
  GEVWS_LB_SMALL_BATCH=0 run mk_dev_$rnd gev_amd/ws_loopback --conns 100 --loops 1 --msg 128 --seconds 3 --client-threads 2
  run cpu_$rnd tools/ws_loopback_cpu --conns 100 --loops 1 --msg 128 --seconds 3 --client-threads 2
done
run sm_dev4 gev_amd/ws_loopback --conns 4000 --loops 4 --msg 128 --seconds 3 --client-threads 8
run cpu4 tools/ws_loopback_cpu --conns 4000 --loops 4 --msg 128 --seconds 3 --client-threads 8
