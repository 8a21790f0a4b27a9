#!/bin/bash
# GPU encode tests, then the encode variant A/B per config (ENC_VARIANTS, default 0,1).
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_encode.py -q -p no:cacheprovider -x > $OUT/enc_tests.log 2>&1
rc=$?; tail -3 $OUT/enc_tests.log; [ $rc -eq 0 ] || exit $rc
for c in ${ENC_CONFIGS:-c3 c2 c4 c5}; do
  timeout -k 10 400 python tools/bench_encode.py --config $c --variants ${ENC_VARIANTS:-0,1} --rounds 3 --reps 5 \
    > $OUT/enc_ab_$c.log 2> $OUT/enc_ab_$c.err || { tail -5 $OUT/enc_ab_$c.err; exit 1; }
  cat $OUT/enc_ab_$c.log
done
