#!/bin/bash
# Sanity pass after a rebuild: GPU parity suite, smoke, default bench, C4 bench.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.err; return $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread; rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 400 python bench.py --cpu-seconds 4 || exit $?
cat $OUT/bench.log
run bench_c4 400 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu || exit $?
cat $OUT/bench_c4.log
