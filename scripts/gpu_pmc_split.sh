#!/bin/bash
# HBM traffic by request size: FETCH_SIZE on gfx950 tallies 128-B read
# requests at 64 B (TCC_BUBBLE), so it is only calibrated for wide streaming
# reads.  This pass counts the L2->fabric read requests of each size directly
# (TCC_EA0_RDREQ_32B / _64B / _128B, 4 TCC counters = one pass) and the write
# requests (TCC_EA0_WRREQ / _64B) plus L2 hits/misses in a second pass, so
# read bytes = 32*n32 + 64*n64 + 128*n128 for every kernel whatever its access
# pattern.  Then a kernel trace of the same command.
#   CONFIGS="c4 c3" BENCH_ARGS="..." PREFIX=split bash scripts/gpu_pmc_split.sh
# PROG replaces bench.py and its arguments (e.g. PROG="tools/bench_encode.py
# --config c4 --rounds 1 --reps 2"; CONFIGS then only names the output);
# NO_TRACE=1 skips the kernel trace.
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for CFG in ${CONFIGS:-c4}; do
  P=$OUT/${PREFIX:-split}_$CFG
  ARGS="$R/bench.py --config $CFG --steps ${STEPS:-3} --warmup 1 --no-cpu --copy-reps 0 ${BENCH_ARGS}"
  [ -n "$PROG" ] && ARGS="$R/$PROG"
  echo "== $CFG read split"
  timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    -d ${P}_rd -o bench --output-format csv -- python3 $ARGS > ${P}_rd.log 2>&1
  rc=$?; echo "rd rc=$rc"; tail -1 ${P}_rd.log; [ $rc -eq 0 ] || exit $rc
  echo "== $CFG write split + L2"
  timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum \
    -d ${P}_wr -o bench --output-format csv -- python3 $ARGS > ${P}_wr.log 2>&1
  rc=$?; echo "wr rc=$rc"; tail -1 ${P}_wr.log; [ $rc -eq 0 ] || exit $rc
  [ -n "$NO_TRACE" ] && continue
  echo "== $CFG trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${P}_trace -o bench --output-format csv \
    -- python3 $ARGS > ${P}_trace.log 2>&1
  rc=$?; echo "trace rc=$rc"; tail -1 ${P}_trace.log; [ $rc -eq 0 ] || exit $rc
done
