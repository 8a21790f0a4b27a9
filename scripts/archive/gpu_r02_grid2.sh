#!/bin/bash
# Round 2: unmask grid sweep on the C4 mix (full batch and the 8-way share) and C3/C2/C5.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for spec_ in ${SPECS:-c4_--emulate-shard_0/8 c4 c5 c2 c3}; do
  spec=${spec_//_/ }; tag=$(echo $spec_ | tr '/' '_')
  timeout -k 10 600 python tools/ab_unmask.py --config $spec --rounds ${ROUNDS:-3} --reps 3 --variants 0 --grids ${GRIDS:-1024,2048,3072,4096,6144} \
    > $OUT/grid2_$tag.json 2> $OUT/grid2_$tag.err || { echo "$spec failed"; tail -3 $OUT/grid2_$tag.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/grid2_$tag.json'))
print('$spec', d.get('stream_copy_ceiling'))
for v in d['variants']: print('   ', v.get('grid'), v['unmask_ms_median'], v['GBps'])"
done
