#!/bin/bash
# Round 2: split walk cost breakdown -- split lanes off, on, on with the
# guesses dropped (mode 1: sync cost + serial walk), on with no guesses
# (mode 2: the split kernel's serial walk alone).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 $OUT/$name.err; return $rc; }
B="python bench.py --steps 10 --warmup 2 --no-cpu --copy-reps 0"
: > $OUT/split_modes.jsonl
for spec_ in ${SPECS:-c4_--emulate-shard_0/8 c2}; do
  spec=${spec_//_/ }
  for m in ${MODES:-1:0 0:0 0:1 0:2}; do
    sl=${m%%:*}; md=${m##*:}
    run sm 300 $B --config $spec --split-lanes $sl --split-mode $md ${EXTRA} || exit $?
    python -c "
import json,sys; d=json.loads(open('$OUT/sm.log').read().strip().splitlines()[-1])
r={'spec':'$spec','split_lanes':$sl,'mode':$md,'ms_per_step':d['ms_per_step'],**d['phases_ms']}
print(json.dumps(r)); open('$OUT/split_modes.jsonl','a').write(json.dumps(r)+'\n')"
  done
done
