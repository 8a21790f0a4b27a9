#!/bin/bash
# Round 2 A/B: pipelined streaming runs (C3), 4-tile pipelined window (C1/C2/C4/C5),
# non-temporal walk header loads (C4).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 $OUT/$name.err; return $rc; }
run pytest_var 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "variant"; rc=$?; tail -2 $OUT/pytest_var.log; [ $rc -eq 0 ] || exit $rc
show() { python -c "
import json; d=json.load(open('$OUT/ab_$1.log'))
print('$1', d['stream_copy_ceiling'])
for v in d['variants']: print('  ', v['variant'], v['unmask_ms_median'], v['GBps'], v['name'][:70])"; }
run ab_c3 900 python tools/ab_unmask.py --config c3 --rounds 4 --reps 3 --variants 0,8,9 --grids 0 && show c3 || exit 1
for c in c1 c2 c4 c5; do run ab_$c 600 python tools/ab_unmask.py --config $c --rounds 4 --reps 3 --variants 0,1,7 --grids 0 && show $c || exit 1; done
WALKS="0 1 5" SPECS="c4" bash scripts/gpu_r02_walk.sh 2>&1 | grep spec
