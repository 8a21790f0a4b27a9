#!/bin/bash
# Round 2, split walk: the whole GPU suite, the stage lines C1-C5, the C4
# strong-scaling projection (rank 0's LPT share of a 2/4/8-way split, auto
# split choice) and a rocprofv3 kernel trace of the 8-way share.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
export TMPDIR=/tmp
bash scripts/gpu_r02_full.sh || exit 1
: > $OUT/shard_proj.jsonl
bash scripts/gpu_shard_proj.sh || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/split_trace -o bench --output-format csv \
  -- python bench.py --config c4 --emulate-shard 0/8 --steps 10 --warmup 2 --no-cpu --copy-reps 0 \
  > $OUT/split_trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/split_trace.log; exit 1; }
tail -1 $OUT/split_trace.log
