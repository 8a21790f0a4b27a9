#!/bin/bash
# Unmask variant parity, then the interleaved unmask A/B (UNMASK_AB) per config.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "unmask_variant or small_frame or golden or c4_full" > $OUT/pytest_um.log 2>&1
rc=$?; tail -3 $OUT/pytest_um.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-c4 c5 c2 c1 c3}; do
  timeout -k 10 600 python tools/ab_unmask.py --config $c --rounds ${ROUNDS:-4} --reps 3 --variants ${UNMASK_AB:-0,11} --grids 0 \
    > $OUT/umab_$c.log 2> $OUT/umab_$c.err || { tail -5 $OUT/umab_$c.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/umab_$c.log'))
print('$c copy', d['stream_copy_ceiling'])
for v in d['variants']: print('  ', v['variant'], v['unmask_ms_median'], v['GBps'], v['name'][:50])"
done
