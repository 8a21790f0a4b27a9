#!/bin/bash
# Round 2: spill-free unmask / encode (fresh_tid) -- variant parity, unmask A/B
# per config, request-size PMC split on C4, encode timings.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -2 $OUT/$name.err; return $rc; }
run pytest_variants 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_encode.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "variant or encode"; rc=$?; tail -3 $OUT/pytest_variants.log; [ $rc -eq 0 ] || exit $rc
for c in c4 c5 c2 c1 c3; do
  run ab_$c 600 python tools/ab_unmask.py --config $c --rounds 4 --reps 3 --variants ${VARIANTS:-0,1,2} --grids 0 || exit $?
  python -c "
import json; d=json.load(open('$OUT/ab_$c.log'))
print('$c', d['stream_copy_ceiling'])
for v in d['variants']: print('  ', v['variant'], v['unmask_ms_median'], v['GBps'], v['name'][:60])"
done
CONFIGS=c4 PREFIX=splitnospill bash scripts/gpu_pmc_split.sh || exit $?
for c in c4 c2 c5; do run enc_$c 600 python tools/bench_encode.py --config $c --reps 5 || exit $?; tail -c 600 $OUT/enc_$c.log; echo; done
