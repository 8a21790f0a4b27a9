#!/bin/bash
# Round 2: record pass with 8 entry rounds per load (emit variant 3) vs the default (4), alternating.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
: > $OUT/emit_u_ab.jsonl
for spec_ in ${SPECS:-c4 c4_--emulate-shard_0/8 c2 c1 c5}; do
  spec=${spec_//_/ }
  for ev in 0 3 3 0; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --copy-reps 0 --config $spec --emit-variant $ev > $OUT/eu.log 2> $OUT/eu.err || { tail -3 $OUT/eu.err; exit 1; }
    python -c "
import json; d=json.loads(open('$OUT/eu.log').read().strip().splitlines()[-1])
r={'spec':'$spec','emit_variant':$ev,'ms_per_step':d['ms_per_step'],**d['phases_ms']}
print(json.dumps(r)); open('$OUT/emit_u_ab.jsonl','a').write(json.dumps(r)+'\n')"
  done
done
