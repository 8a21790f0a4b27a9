#!/bin/bash
# rocprofv3 kernel trace of the outbound encode bench (per-kernel split).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-c4 c2}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_enc_$c -o enc --output-format csv \
    -- python3 $R/tools/bench_encode.py --config $c --reps 5 > $OUT/prof_enc_$c.log 2>&1
  rc=$?; echo "enc $c rc=$rc"; tail -1 $OUT/prof_enc_$c.log; [ $rc -eq 0 ] || exit $rc
done
