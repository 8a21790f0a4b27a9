#!/bin/bash
# Round 2: grouped record pass (emit variant 0) vs one wave per connection (1).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 $OUT/$name.err; return $rc; }
run pytest_emit 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "emit or walk or c4_full or random or golden or unordered"; rc=$?; tail -2 $OUT/pytest_emit.log; [ $rc -eq 0 ] || exit $rc
: > $OUT/emit_ab.jsonl
for spec_ in ${SPECS:-c1 c2 c4 c4_--emulate-shard_0/8 c5 c3}; do
  spec=${spec_//_/ }
  for ev in ${EMITS:-0 1 0 1}; do
    run eab 300 python bench.py --steps 10 --warmup 2 --no-cpu --copy-reps 0 --config $spec --emit-variant $ev || exit $?
    python -c "
import json; d=json.loads(open('$OUT/eab.log').read().strip().splitlines()[-1])
r={'spec':'$spec','emit':$ev,'ms_per_step':d['ms_per_step'],**d['phases_ms']}
print(json.dumps(r)); open('$OUT/emit_ab.jsonl','a').write(json.dumps(r)+'\n')"
  done
done
