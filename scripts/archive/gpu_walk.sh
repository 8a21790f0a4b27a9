#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.err; return $rc; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for c in c4 c5 c2 c3; do
run walk_$c 600 python bench.py --config $c --steps 10 --warmup 2 --no-cpu || exit $?
python -c "
import json; d=json.loads(open('$OUT/walk_$c.log').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d['roofline']['pipeline_frac'])"
done
