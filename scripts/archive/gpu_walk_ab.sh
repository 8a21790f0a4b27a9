#!/bin/bash
# Walk variants: parity tests, then bench per config with the speculative walk
# (default) and the plain chain walk (bench.py --walk-variant 1).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.err; return $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread; rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c2 c4 c5 c3}; do
  for wv in 0 1; do
    run walk_${c}_$wv 500 python bench.py --config $c --walk-variant $wv --steps 10 --warmup 2 --no-cpu --copy-reps 0 || exit $?
    python -c "
import json; d=json.loads(open('$OUT/walk_${c}_$wv.log').read().strip().splitlines()[-1]); print('$c walk$wv', d['value'], d['ms_per_step'], d['phases_ms'])"
  done
done
