#!/bin/bash
# v4 (pipelined window) vs v3: variant parity tests, then interleaved A/B per config.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.err; return $rc; }
run pytest_variants 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "variant"; rc=$?; tail -4 $OUT/pytest_variants.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c4 c5 c2 c3}; do
  run ab_$c 600 python tools/ab_unmask.py --config $c --rounds 4 --reps 3 --variants ${VARIANTS:-0,1} --grids 0 || exit $?
  python -c "
import json; d=json.load(open('$OUT/ab_$c.log'))
print('$c', d['stream_copy_ceiling'])
for v in d['variants']: print('  ', v['variant'], v['unmask_ms_median'], v['GBps'], v['name'][:60])"
done
