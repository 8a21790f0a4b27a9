#!/bin/bash
# bench.py with 1 vs 2 batches in flight (two contexts on two streams), per config.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for c in ${CONFIGS:-c4 c5 c2 c3}; do
  for m in ${INFLIGHT:-1 2 1 2}; do
    timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 --no-cpu --copy-reps 0 --inflight $m \
      > $OUT/infl_${c}_$m.log 2> $OUT/infl_${c}_$m.err || { echo "bench $c $m failed"; tail -5 $OUT/infl_${c}_$m.err; exit 1; }
    python -c "
import json; d=json.loads(open('$OUT/infl_${c}_$m.log').read().strip().splitlines()[-1])
print('$c', 'inflight', $m, 'value', d['value'], 'ms_step', d['ms_per_step'], 'phases', d['phases_ms'])"
    tail -1 $OUT/infl_${c}_$m.log >> $OUT/infl_${c}.jsonl
  done
done
