#!/bin/bash
# GPU session: parity tests, then bench on every config and the host-inclusive rate.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.err; cat $OUT/$name.log | tail -c 3000; return $rc; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x; rc=$?; [ $rc -le 1 ] || exit $rc
run bench_c3 300 python bench.py --steps 20 --warmup 3 --no-cpu || exit $?
run bench_c2 300 python bench.py --config c2 --steps 50 --warmup 5 --no-cpu || exit $?
run bench_c5 300 python bench.py --config c5 --steps 50 --warmup 5 --no-cpu || exit $?
run bench_c4 600 python bench.py --config c4 --steps 10 --warmup 2 --no-cpu || exit $?
run host_incl 600 python tools/host_inclusive.py --gib 8 || exit $?
