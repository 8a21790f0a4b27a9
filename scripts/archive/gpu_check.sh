#!/bin/bash
# GPU session: parity tests, smoke, A/B of unmask variants, bench, rocprof.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.err
  return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x
rc=$?; tail -15 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
step smoke 180 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step ab 600 python tools/ab_unmask.py --rounds 5 --reps 3 --grids 0 || exit $?
cat $OUT/ab.log
step bench 400 python bench.py --steps 20 --warmup 3 || exit $?
cat $OUT/bench.log
