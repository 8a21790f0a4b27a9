#!/bin/bash
# HBM bytes (FETCH_SIZE / WRITE_SIZE, separate passes) of the encode bench.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C=${CFG:-c4}
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/pmc_enc_$P -o enc --output-format csv \
    -- python3 $R/tools/bench_encode.py --config $C --reps 1 --rounds 1 > $OUT/pmc_enc_$P.log 2>&1
  rc=$?; echo "$P rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
