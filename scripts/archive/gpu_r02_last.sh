#!/bin/bash
# Round 2, last check of the tree as committed: whole GPU suite, smoke, the
# default bench line, stage lines.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 $OUT/$name.err; return $rc; }
SPECS="${SPECS:-c1 c2 c3 c4 c4_--emulate-shard_0/8 c5}" bash scripts/gpu_r02_full.sh || exit 1
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench 600 python bench.py || exit 1
tail -c 600 $OUT/bench.log
