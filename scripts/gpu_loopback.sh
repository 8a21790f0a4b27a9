#!/bin/bash
# GPU parity suite, then the live loopback echo server (host ingress, C1
# shape: masked 128 B text frames, binary echoes) at a few connection counts.
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.err
  return $rc
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x
  rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
export GEV_LOG_LEVEL=FATAL
for spec in ${LOOPBACK_SPECS:-"100:1:2" "1000:1:4" "4000:1:8" "4000:2:8"}; do
  IFS=: read C L T <<< "$spec"
  step loop_${C}_${L} 120 $R/gev_amd/ws_loopback --conns $C --loops $L --client-threads $T --msg 128 --seconds 5 || exit $?
  cat $OUT/loop_${C}_${L}.log
done
