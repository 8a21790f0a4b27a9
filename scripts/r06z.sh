# round 6: where a live pass's ~9 us goes (tools/live_pass_probe.py): the
# C1 pass shape (100 connections x one masked 128-byte frame) with input and
# outputs in device memory or mapped pinned host memory, launched or written
# into the context's own AQL queue.  Predicted: the kernel ~4 us with
# everything in device memory, +2-3 us for host input (the staged read), +1-2
# us for host outputs (the write-back before the signal); post -> signal
# ~3 us above the kernel's own time (dispatch + the host's spin).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/live_pass_probe.py --reps 300 > gpurun_out/r06z_live_pass_probe.jsonl 2> gpurun_out/r06z.err &&
GEVWS_PHASE_TICKS=1 timeout -k 10 300 python -u tools/live_pass_probe.py --reps 300 > gpurun_out/r06z_live_pass_phases.jsonl 2>> gpurun_out/r06z.err
# (first run: kernel 8.0 us with input and outputs in device memory, 9.3 with
# host input; post -> signal 18-20 us launched, 21.5-23 us direct -- so a
# second run stamps the kernel's phases, GEVWS_PHASE_TICKS=1: staged / parsed /
# scanned / stored)
