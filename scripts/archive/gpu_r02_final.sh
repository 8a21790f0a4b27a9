#!/bin/bash
# Round-2 final evidence: whole GPU suite, smoke, the default bench line (CPU
# baselines, copy ceiling by load kind), stage lines C1-C5 + C4 rank-0 share,
# C3 / C4 request-size PMC split + kernel traces (PREFIX=r02f).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -5 $OUT/$name.err; return $rc; }
bash scripts/gpu_r02_full.sh || exit 1
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench 600 python bench.py || exit 1
tail -c 1500 $OUT/bench.log
CONFIGS="c3 c4" PREFIX=${PREFIX:-r02f} STEPS=5 bash scripts/gpu_pmc_split.sh || exit 1
