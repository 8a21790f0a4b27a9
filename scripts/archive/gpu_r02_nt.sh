#!/bin/bash
# Non-temporal streaming loads: unmask + encode parity, interleaved A/Bs, the
# default bench line (its copy ceiling now uses the same loads).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
CONFIGS="c3 c4 c5 c2 c1" UNMASK_AB=0,12 ROUNDS=4 bash scripts/gpu_r02_unmask_ab.sh || exit 1
ENC_CONFIGS="c3 c4 c2" ENC_VARIANTS=0,8 bash scripts/gpu_r02_encode.sh || exit 1
timeout -k 10 600 python bench.py --no-cpu > $OUT/bench_nt.log 2> $OUT/bench_nt.err || exit 1
tail -1 $OUT/bench_nt.log | cut -c1-600
