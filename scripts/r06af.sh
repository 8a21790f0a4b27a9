# round 6: the C4 8-way share's step is 1.396-1.398 ms against the review's
# 1.38 target; its unmask (0.91 ms, 5.3 TB/s against the full batch's 5.8)
# is the largest phase.  Interleaved A/B of the unmask grid on that share
# (auto = the wide grid, 32 workgroups per CU, after a mixed batch) against
# 8 / 16 / 64 per CU, plus the walk's lanes-per-CU budget.  Predicted: no
# grid more than 2 % faster (the share's unmask is fill / drain bound, like
# C2 / C5), i.e. the 1.40 ms stands as the floor of this design.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_decode.py --workloads 'c4@0/8' \
  --configs 'auto:;g8:UNMASK_GRID=2048;g16:UNMASK_GRID=4096;g64:UNMASK_GRID=16384;lpc256:SPLIT_LANES_PER_CU=256;lpc1k:SPLIT_LANES_PER_CU=1024' \
  --rounds 4 --reps 3 --out gpurun_out/r06af_share_ab.jsonl > gpurun_out/r06af.log 2>&1
