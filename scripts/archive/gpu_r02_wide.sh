#!/bin/bash
# Round 2: the unmask's wide grid -- split/grid tests, then stage lines with
# the auto choices (C4 8-way share, C4, C2, C5, C1, C3).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 $OUT/$name.err; return $rc; }
run pytest_split 600 python -u -m pytest tests/test_gpu_split.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread; rc=$?; tail -3 $OUT/pytest_split.log; [ $rc -eq 0 ] || exit $rc
SPECS="${SPECS:-c4_--emulate-shard_0/8 c4_--emulate-shard_0/4 c4_--emulate-shard_0/2 c4 c2 c5 c1 c3}" bash scripts/gpu_r02_full_steps.sh
