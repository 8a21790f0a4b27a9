# round 6: r06o showed the C4 encode's traffic equal to the unmask's (40.96
# against 40.68 GB a launch) but its 4 launches at 7.63 / 7.69 / 7.21 / 7.11 ms
# against the unmask's steady 7.37-7.44: the first two follow seconds of
# host-side set-up with the GPU idle.  Predicted: with untimed encodes first,
# k_encode6 settles at ~7.1-7.2 ms = 0.96-0.98 x the same process's unmask
# on any box, and without them (--warmup 0) the first round is ~7 % slower --
# the clocks' ramp after idle, not the kernel, being the box-dependent term.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_encode.py --config c4 --rounds 5 --reps 3 --warmup 0 > gpurun_out/r06p_encode.jsonl 2>gpurun_out/r06p_encode.err &&
timeout -k 10 300 python tools/bench_encode.py --config c4 --rounds 5 --reps 3 --warmup 3 >> gpurun_out/r06p_encode.jsonl 2>>gpurun_out/r06p_encode.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06p_trace -o bench --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/tools/bench_encode.py --config c4 --rounds 1 --reps 3 --warmup 3 --decode-reps 3 \
  >> $GRAFT_REPO_ROOT/gpurun_out/r06p_encode.jsonl 2>>$GRAFT_REPO_ROOT/gpurun_out/r06p_encode.err
