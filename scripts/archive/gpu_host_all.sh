#!/bin/bash
# Host-side paths with the current kernels: host-inclusive bulk decode sweep
# (pinned H2D -> decode -> D2H) and the live loopback echo server.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 600 python tools/host_inclusive.py --gib 8 --reps 2 --sweep 32:2,64:2,64:3,128:2,128:3,256:2 > $OUT/host_sweep.log 2> $OUT/host_sweep.err
rc=$?; echo host rc=$rc; tail -3 $OUT/host_sweep.err; cat $OUT/host_sweep.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 LOOPBACK_SPECS="100:1:2 1000:1:4 4000:4:8 8000:6:12" bash scripts/gpu_loopback.sh
