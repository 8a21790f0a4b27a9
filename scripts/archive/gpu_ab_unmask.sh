#!/bin/bash
# GPU parity suite, then an interleaved A/B of unmask variants (VARIANTS) per config.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c4 c2 c5 c3}; do
  timeout -k 10 600 python tools/ab_unmask.py --config $c --rounds ${ROUNDS:-5} --reps 3 --variants ${VARIANTS:-0,1} --grids 0 \
    > $OUT/abu_$c.log 2> $OUT/abu_$c.err || { tail -5 $OUT/abu_$c.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/abu_$c.log'))
for v in d['variants']: print('$c', v['variant'], v['unmask_ms_median'], v['GBps'], v['name'][:40])"
done
