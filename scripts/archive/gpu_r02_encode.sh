#!/bin/bash
# Encode parity (all variants, queue-capacity windows), then the interleaved
# encode A/B per config (ENC_VARIANTS, ENC_CONFIGS).
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/enc_tests.log 2>&1
rc=$?; tail -5 $OUT/enc_tests.log; [ $rc -eq 0 ] || exit $rc
for c in ${ENC_CONFIGS:-c4 c2 c5 c3}; do
  timeout -k 10 300 python tools/bench_encode.py --config $c --variants ${ENC_VARIANTS:-0,5,4} --rounds 3 --reps 5 \
    > $OUT/enc_ab_$c.log 2> $OUT/enc_ab_$c.err || { tail -5 $OUT/enc_ab_$c.err; exit 1; }
  grep -v '^ *$' $OUT/enc_ab_$c.log | tail -4
done
if [ -n "$ENC_TRACE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd $R
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/enc_trace_c4 -o enc -- \
    python tools/bench_encode.py --config c4 --variants $ENC_TRACE --rounds 1 --reps 5 > $OUT/enc_trace_c4.log 2>&1 || exit 1
fi
