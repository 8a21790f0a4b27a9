#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.err; return $rc; }
run grid_c3 600 python tools/ab_unmask.py --config c3 --rounds 4 --reps 2 --variants 0 --grids 256,384,512,768,1024 || exit $?
run grid_c4 900 python tools/ab_unmask.py --config c4 --rounds 3 --reps 2 --variants 0 --grids 256,512,1024,2048 || exit $?
run grid_c2 300 python tools/ab_unmask.py --config c2 --rounds 5 --reps 5 --variants 0 --grids 256,512,1024,2048 || exit $?
run grid_c5 300 python tools/ab_unmask.py --config c5 --rounds 5 --reps 5 --variants 0 --grids 256,512,1024,2048 || exit $?
for f in grid_c3 grid_c4 grid_c2 grid_c5; do python -c "
import json; d=json.load(open('$OUT/$f.log')); print('$f', d['workload'], d['copy_ceiling'])
for v in d['variants']: print('  ', v['grid'], v['unmask_ms_median'], v['unmask_ms_min'], v['GBps'], v['frac_of_8TBps'])"; done
