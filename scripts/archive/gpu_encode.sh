#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.err; tail -c 1500 $OUT/$name.log; return $rc; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x; rc=$?; [ $rc -le 1 ] || exit $rc
run enc_c3 600 python tools/bench_encode.py --config c3 || exit $?
run enc_c2 300 python tools/bench_encode.py --config c2 || exit $?
run enc_c5 300 python tools/bench_encode.py --config c5 || exit $?
run enc_c4 600 python tools/bench_encode.py --config c4 --reps 5 || exit $?
