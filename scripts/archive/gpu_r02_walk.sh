#!/bin/bash
# Round 2: the one-wave-per-connection span walk (k_walk_span) against the
# lane walk -- walk-variant parity first, then per-config phase timings.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 $OUT/$name.err; return $rc; }
run pytest_walk 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "walk or c4_full or 4gib or c5 or c4_power"; rc=$?; tail -3 $OUT/pytest_walk.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 10 --warmup 2 --no-cpu --copy-reps 0"
: > $OUT/walk_ab.jsonl
# specs: words joined by "_" (e.g. c4_--emulate-shard_0/8)
for spec_ in ${SPECS:-c4_--emulate-shard_0/8 c4_--emulate-shard_0/4 c4_--emulate-shard_0/2 c4 c5 c2 c1 c3}; do
  spec=${spec_//_/ }
  for wv in ${WALKS:-3 6 7}; do
    run wab 300 $B --config $spec --walk-variant $wv ${EXTRA} || exit $?
    python -c "
import json,sys; d=json.loads(open('$OUT/wab.log').read().strip().splitlines()[-1])
r={'spec':'$spec','walk':$wv,'ms_per_step':d['ms_per_step'],**d['phases_ms']}
print(json.dumps(r)); open('$OUT/walk_ab.jsonl','a').write(json.dumps(r)+'\n')"
  done
done
if [ -n "$UNMASK_AB" ]; then
  for c in c4 c5 c2; do
    run ab_$c 600 python tools/ab_unmask.py --config $c --rounds 4 --reps 3 --variants $UNMASK_AB --grids 0 || exit $?
    python -c "
import json; d=json.load(open('$OUT/ab_$c.log'))
print('$c', d['stream_copy_ceiling'])
for v in d['variants']: print('  ', v['variant'], v['unmask_ms_median'], v['GBps'], v['name'][:60])"
  done
fi
