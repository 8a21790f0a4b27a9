#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.err; return $rc; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
run auto_c3 600 python tools/ab_unmask.py --config c3 --rounds 4 --reps 2 --variants 0 --grids 0,256,1024 || exit $?
run auto_c4 900 python tools/ab_unmask.py --config c4 --rounds 3 --reps 2 --variants 0 --grids 0,1024 || exit $?
run bench_c3 300 python bench.py --steps 20 --warmup 3 || exit $?
tail -c 3000 $OUT/bench_c3.log
run enc_c3 600 python tools/bench_encode.py --config c3 || exit $?
tail -c 600 $OUT/enc_c3.log
for f in auto_c3 auto_c4; do python -c "
import json; d=json.load(open('$OUT/$f.log')); print('$f', d['workload'], d['copy_ceiling'])
for v in d['variants']: print('  ', v['grid'], v['unmask_ms_median'], v['unmask_ms_min'], v['GBps'], v['frac_of_8TBps'])"; done
