#!/bin/bash
# C4 strong-scaling projection on one GPU: the full batch, then rank 0's LPT
# share of a 2-, 4- and 8-way split (bench.py --emulate-shard).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for sh in 0/1 0/2 0/4 0/8 7/8; do
  tag=$(echo $sh | tr / _)
  timeout -k 10 400 python bench.py --config ${CFG:-c4} --steps 10 --warmup 2 --no-cpu --copy-reps 0 --emulate-shard $sh \
    > $OUT/shard_$tag.log 2> $OUT/shard_$tag.err || { echo "shard $sh failed"; tail -5 $OUT/shard_$tag.err; exit 1; }
  python -c "
import json; d=json.loads(open('$OUT/shard_$tag.log').read().strip().splitlines()[-1])
print('$sh', d['ms_per_step'], d['value'], d['config']['frames_per_gpu'], d['config']['connections_per_gpu'], d['phases_ms'])"
  tail -1 $OUT/shard_$tag.log >> $OUT/shard_proj.jsonl
done
