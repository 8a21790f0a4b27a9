#!/bin/bash
# Interleaved A/B of the header walk variants (0 = speculative, 1 = plain) per
# config, with the default unmask kernel; parity suite first.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.err; return $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread; rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c2 c5 c4 c3}; do
  run abw_$c 600 python tools/ab_unmask.py --config $c --rounds 5 --reps 3 --variants 0 --grids 0 --walk-variants ${WALKS:-0,1} || exit $?
  python -c "
import json; d=json.load(open('$OUT/abw_$c.log'))
for v in d['variants']: print('$c', 'walk', v['walk_variant'], 'count', v['walk_count_ms'], 'emit', v['walk_emit_ms'], 'unmask', v['unmask_ms_median'])"
done
