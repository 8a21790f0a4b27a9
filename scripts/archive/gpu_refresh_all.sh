#!/bin/bash
# Refresh every committed measurement with the current defaults: full GPU
# parity suite, smoke, the default bench line (C3, with cpu_baseline), bench
# lines for C2/C4/C5, then rocprofv3 trace + PMC passes for C3 and C4.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.err; return $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 500 python bench.py || exit $?
cat $OUT/bench.log
for c in c2 c4 c5; do
  run bench_$c 500 python bench.py --config $c --steps 10 --warmup 2 --no-cpu || exit $?
  tail -c 600 $OUT/bench_$c.log; echo
done
PREFIX=prof_c3 bash scripts/gpu_profile.sh || exit $?
PREFIX=prof_c4 BENCH_ARGS="--config c4" STEPS=5 bash scripts/gpu_profile.sh || exit $?
# outbound encode and the device server step (decode + dispatch + encode)
for c in c3 c2 c5 c4; do
  run enc_$c 600 python tools/bench_encode.py --config $c --reps 5 || exit $?
done
for c in c1 c2 c5 c3; do
  run srv_$c 600 python tools/bench_server.py --config $c --reps 5 || exit $?
done
