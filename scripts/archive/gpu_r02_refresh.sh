#!/bin/bash
# Round-2 evidence: smoke, the default bench line (with the all-cores CPU
# baseline), then for C3 and C4 a rocprofv3 kernel trace + the request-size
# PMC passes (scripts/gpu_pmc_split.sh) and the loopback pair (C1).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 $OUT/$name.err; return $rc; }
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 600 python bench.py || exit $?
tail -c 3000 $OUT/bench.log
CONFIGS="${CONFIGS:-c3 c4}" PREFIX=r02 STEPS=5 bash scripts/gpu_pmc_split.sh || exit $?
run lb_dev 120 gev_amd/ws_loopback --conns 100 --loops 1 --msg 128 --seconds 3 --client-threads 2 || exit $?
run lb_cpu 120 tools/ws_loopback_cpu --conns 100 --loops 1 --msg 128 --seconds 3 --client-threads 2 || exit $?
run lb_dev4 120 gev_amd/ws_loopback --conns 4000 --loops 4 --msg 128 --seconds 3 --client-threads 8 || exit $?
run lb_cpu4 120 tools/ws_loopback_cpu --conns 4000 --loops 4 --msg 128 --seconds 3 --client-threads 8 || exit $?
cat $OUT/lb_*.log
