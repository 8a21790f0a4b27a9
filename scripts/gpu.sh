#!/bin/bash
# One parameterised runner for every GPU measurement (replaces the round-1/2
# single-use scripts).  Each argument is one step; steps run in order, each
# under its own time limit, and the first failure ends the run (no GPU work
# after a fault, abort or timeout).
#
#   bash scripts/gpu.sh 'test tests/test_gpu_parity.py' \
#                       'bench c4i2 --config c4 --inflight 2' \
#                       'prof c4 --config c4 --steps 5' \
#                       'pmc c4_rd TCC_EA0_RDREQ_32B,TCC_EA0_RDREQ_64B -- --config c4 --steps 3' \
#                       'py tools/host_inclusive.py --out gpurun_out/x.json'
#
# test  <pytest args>      python -m pytest -x -v (thread timeout per test)
# bench <tag> <bench args> bench.py --no-cpu --copy-reps 0 (unless given) --steps 10 --warmup 2 (unless
#                          given); the JSON line, tagged, appended to $OUT/${JSONL:-bench}.jsonl
# full  <tag> <bench args> bench.py exactly as given (the contract line: CPU legs, copy ceiling)
# prof  <tag> <bench args> the bench under rocprofv3 --kernel-trace --stats -> $OUT/prof_<tag>/
# pmc   <tag> <ctrs> -- <bench args>  one rocprofv3 --pmc pass (counters comma-separated)
# py    <args>             python <args>
# pyprof <tag> <args>      python <args> under rocprofv3 --kernel-trace --stats -> $OUT/prof_<tag>/
# sh    <command line>     bash -c <command line> (e.g. the loopback binaries)
# Time limits: STEP_TIMEOUT (default 300 s) per step, 900 s for `test`.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  set -- $step
  kind=$1; shift
  to=${STEP_TIMEOUT:-300}
  log=$OUT/step$n.log; err=$OUT/step$n.err
  echo "== [$n] $step"
  case $kind in
    test)
      to=${TEST_TIMEOUT:-900}
      timeout -k 10 $to python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread "$@" \
        > $log 2> $err; rc=$?
      tail -4 $log ;;
    bench|full)
      tag=$1; shift
      extra=""
      if [ $kind = bench ]; then
        [[ " $* " == *" --steps "* ]] || extra="$extra --steps 10"
        [[ " $* " == *" --warmup "* ]] || extra="$extra --warmup 2"
        [[ " $* " == *" --copy-reps "* ]] || extra="$extra --copy-reps 0"
        [[ " $* " == *" --no-cpu"* || " $* " == *" --cpu-seconds "* ]] || extra="$extra --no-cpu"
      fi
      timeout -k 10 $to python -u bench.py "$@" $extra > $log 2> $err; rc=$?
      if [ $rc -eq 0 ]; then
        python - "$log" "$tag" "$OUT/${JSONL:-bench}.jsonl" "$*$extra" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d["tag"], d["args"] = sys.argv[2], sys.argv[4]
open(sys.argv[3], "a").write(json.dumps(d) + "\n")
w = d.get("walk", {})
print(sys.argv[2], "ms/step", d["ms_per_step"], "GiB/s", d["value"], "phases", d["phases_ms"],
      "walk", w, "frac", d["roofline"]["frac"], "copy", d["roofline"].get("copy_ceiling_by_load"))
PY
      fi ;;
    prof)
      tag=$1; shift
      timeout -k 10 $to rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$tag -o $tag -- \
        python -u bench.py --no-cpu --copy-reps 0 "$@" > $log 2> $err; rc=$?
      [ $rc -eq 0 ] && tail -c 600 $log ;;
    pmc)
      tag=$1; ctrs=$2; shift 3
      timeout -s KILL 120 rocprofv3 --pmc ${ctrs//,/ } -d $OUT/pmc_$tag -o $tag -- \
        python -u bench.py --no-cpu --copy-reps 0 "$@" > $log 2> $err; rc=$? ;;
    py)
      timeout -k 10 $to python -u "$@" > $log 2> $err; rc=$?
      tail -c 1500 $log ;;
    sh)
      timeout -k 10 $to bash -c "$*" > $log 2> $err; rc=$?
      tail -c 1500 $log ;;
    pyprof)
      tag=$1; shift
      timeout -k 10 $to rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$tag -o $tag -- python -u "$@" > $log 2> $err
      rc=$?
      [ $rc -eq 0 ] && tail -c 600 $log ;;
    *)
      echo "unknown step kind: $kind"; exit 2 ;;
  esac
  echo "[$n] rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $err; tail -20 $log; exit $rc; fi
done
