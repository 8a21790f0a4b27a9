#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 600 python tools/ab_unmask.py --rounds 5 --reps 3 --variants 0,2,3,4,5,6 --grids 512,768,1024,1536 > $OUT/ab2.log 2> $OUT/ab2.err
rc=$?; echo "ab rc=$rc"; tail -2 $OUT/ab2.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_unmask.py --rounds 3 --reps 3 --variants 0,3 --grids 1024 --align-payload > $OUT/ab_aligned.log 2> $OUT/ab_aligned.err
rc=$?; echo "ab aligned rc=$rc"; tail -2 $OUT/ab_aligned.err; [ $rc -eq 0 ] || exit $rc
bash $R/scripts/gpu_profile.sh
