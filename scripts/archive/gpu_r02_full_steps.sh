#!/bin/bash
# Round 2: one decode-step line per config (phases), no test suite.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 $OUT/$name.err; return $rc; }
: > $OUT/steps.jsonl
for spec_ in ${SPECS:-c1 c2 c3 c4 c4_--emulate-shard_0/8 c5}; do
  spec=${spec_//_/ }
  run st 300 python bench.py --steps 10 --warmup 2 --no-cpu --copy-reps 3 --config $spec ${EXTRA} || exit $?
  python -c "
import json; d=json.loads(open('$OUT/st.log').read().strip().splitlines()[-1])
r={'spec':'$spec','value':d['value'],'ms_per_step':d['ms_per_step'],**d['phases_ms'],'frac':d['roofline']['frac'],'copy':d['roofline']['copy_ceiling'],'frac_copy':d['roofline']['frac_of_copy_ceiling']}
print(json.dumps(r)); open('$OUT/steps.jsonl','a').write(json.dumps(r)+'\n')"
done
