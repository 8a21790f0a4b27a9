#!/bin/bash
# Round 2: split header walk (k_walk_split) -- its parity tests, then the
# per-config phase timings with GEVWS_TUNE_SPLIT_LANES off (1) / auto (0) /
# forced, alternating order.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 $OUT/$name.err; return $rc; }
run pytest_split 600 python -u -m pytest tests/test_gpu_split.py ${TESTS_EXTRA} -x -q -p no:cacheprovider --timeout 300 --timeout-method thread; rc=$?; tail -3 $OUT/pytest_split.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 10 --warmup 2 --no-cpu --copy-reps 0"
: > $OUT/split_ab.jsonl
for spec_ in ${SPECS:-c4_--emulate-shard_0/8 c4_--emulate-shard_0/4 c4 c2 c5 c3}; do
  spec=${spec_//_/ }
  for sl in ${LANES:-1 0}; do
    run sab 300 $B --config $spec --split-lanes $sl ${EXTRA} || exit $?
    python -c "
import json,sys; d=json.loads(open('$OUT/sab.log').read().strip().splitlines()[-1])
r={'spec':'$spec','split_lanes':$sl,'ms_per_step':d['ms_per_step'],**d['phases_ms']}
print(json.dumps(r)); open('$OUT/split_ab.jsonl','a').write(json.dumps(r)+'\n')"
  done
done
