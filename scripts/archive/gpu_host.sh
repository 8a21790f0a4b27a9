#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python tools/host_inclusive.py --gib 8 --reps 2 --sweep 32:2,64:2,64:3,128:2,128:3,256:3,512:2,512:3,128:4 > $OUT/host_sweep.log 2> $OUT/host_sweep.err
rc=$?; echo rc=$rc; tail -3 $OUT/host_sweep.err; cat $OUT/host_sweep.log
