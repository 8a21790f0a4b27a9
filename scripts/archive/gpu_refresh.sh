#!/bin/bash
# Refresh the committed evidence with the current defaults: GPU parity suite,
# smoke, the default bench line (with cpu_baseline), then the rocprofv3 trace +
# PMC passes of the C3 bench (scripts/gpu_profile.sh).  Any failure ends it.
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name"; timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; tail -3 $OUT/$name.err
  return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x
rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
step smoke 180 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 400 python bench.py || exit $?
cat $OUT/bench.log
bash $R/scripts/gpu_profile.sh
