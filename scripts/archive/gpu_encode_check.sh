#!/bin/bash
# GPU parity suite, then the outbound encode and server-step benches per config.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.err; return $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${ENC_CONFIGS:-c4 c2 c5 c3}; do
  run enc_$c 600 python tools/bench_encode.py --config $c --reps 5 --variants ${ENC_VARIANTS:-0} || exit $?
  tail -c 400 $OUT/enc_$c.log; echo
done
for c in ${SRV_CONFIGS:-c1 c2 c5}; do
  run srv_$c 600 python tools/bench_server.py --config $c --reps 5 || exit $?
  tail -c 400 $OUT/srv_$c.log; echo
done
