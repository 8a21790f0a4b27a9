#!/bin/bash
# Kernel + memory-copy trace of the live loopback server (C1, 100 conns):
# where a device pass's ~80 us go.
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $R
export GEV_LOG_LEVEL=FATAL
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/lbprof -o lb --output-format csv -- \
  $R/gev_amd/ws_loopback --conns 100 --loops 1 --msg 128 --seconds 2 --client-threads 2 > $OUT/lbprof.log 2>&1 || exit 1
tail -2 $OUT/lbprof.log
