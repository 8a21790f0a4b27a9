#!/bin/bash
# Translation misses of the header walk: UTCL1 requests / misses per kernel
# (one --pmc pass per config), C4 whole batch and rank 0's 1/8 share.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for spec in "c4" "c4 --emulate-shard 0/8" "c3"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_sum \
    -d $OUT/tlb_$i -o p --output-format csv -- python3 $R/bench.py --config $spec --steps 2 --warmup 1 --no-cpu --copy-reps 0 \
    > $OUT/tlb_$i.log 2>&1 || { tail -5 $OUT/tlb_$i.log; exit 1; }
done
echo done
