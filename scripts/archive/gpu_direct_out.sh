#!/bin/bash
# Host-inclusive decode, payload D2H copy vs the unmask kernel writing the
# payload straight into mapped pinned host memory (--direct-out).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "mapped_host_arena or golden" > $OUT/direct_test.log 2>&1
rc=$?; tail -5 $OUT/direct_test.log; [ $rc -eq 0 ] || exit $rc
SW=${SWEEP:-16:2,32:2,64:2,32:3}
timeout -k 10 400 python tools/host_inclusive.py --gib 8 --reps 2 --sweep $SW --direct-out > $OUT/direct_sweep.log 2> $OUT/direct_sweep.err
rc=$?; echo direct rc=$rc; tail -3 $OUT/direct_sweep.err; cat $OUT/direct_sweep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/host_inclusive.py --gib 8 --reps 2 --sweep $SW > $OUT/copy_sweep.log 2> $OUT/copy_sweep.err
rc=$?; echo copy rc=$rc; tail -3 $OUT/copy_sweep.err; cat $OUT/copy_sweep.log; exit $rc
