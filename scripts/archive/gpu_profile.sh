#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then one PMC
# pass per counter (FETCH_SIZE, WRITE_SIZE), each in its own run (no trace
# domains combined with --pmc).  Outputs under gpurun_out/${PREFIX:-prof}_*.
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps ${STEPS:-10} --warmup 2 --no-cpu ${BENCH_ARGS}"
echo "== trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/${PREFIX:-prof}_trace -o bench --output-format csv \
  -- python3 $R/bench.py $ARGS > $OUT/${PREFIX:-prof}_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 $OUT/${PREFIX:-prof}_trace.log; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C"
  timeout -k 10 400 rocprofv3 --pmc $C -d $OUT/${PREFIX:-prof}_pmc_$C -o bench --output-format csv \
    -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu ${BENCH_ARGS} > $OUT/${PREFIX:-prof}_pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; tail -2 $OUT/${PREFIX:-prof}_pmc_$C.log; [ $rc -eq 0 ] || exit $rc
done
find $OUT/${PREFIX:-prof}_* -name "*.csv" | head -20
