#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.err; return $rc; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x; rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
run ab_c4 900 python tools/ab_unmask.py --config c4 --rounds 3 --reps 2 --variants 0,2,5 || exit $?
run ab_c5 300 python tools/ab_unmask.py --config c5 --rounds 5 --reps 5 --variants 0,2,5 || exit $?
run ab_c2 300 python tools/ab_unmask.py --config c2 --rounds 5 --reps 5 --variants 0,2,5 || exit $?
run ab_c3 600 python tools/ab_unmask.py --config c3 --rounds 4 --reps 2 --variants 0,2 --grids 512,1024 || exit $?
for f in ab_c4 ab_c5 ab_c2 ab_c3; do python -c "
import json; d=json.load(open('$OUT/$f.log')); print('$f', d['workload'], d['copy_ceiling'])
for v in d['variants']: print('  ', v['variant'], v['grid'], v['name'], v['unmask_ms_median'], v['GBps'], v['frac_of_8TBps'], v['walk_count_ms'], v['walk_emit_ms'])"; done
