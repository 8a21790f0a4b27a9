#!/bin/bash
# The live path's per-pass timeline: the loopback echo
# server, 100 connections on 1 loop (128 B masked frames) and the wsserver
# shape, device decode (passes split in two groups by default, and one pass
# per iteration with GEVWS_LB_SPLIT=0) beside the CPU twin; each line carries
# pass_timeline_us (host select / stage / launch / wait / deliver, and the
# one-launch kernels' GPU time).  Lines -> gpurun_out/${TAG}_loopback_timeline.jsonl
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
export GEV_LOG_LEVEL=FATAL
OUT=gpurun_out/${TAG:-r05}_loopback_timeline.jsonl
run() {  # run <label> <env> <binary> <args>
  local label=$1 envs=$2 bin=$3; shift 3
  env $envs timeout -k 5 60 $bin --seconds ${SECS:-3} "$@" | grep '^{' | \
    python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['label']='$label'; d['env']='$envs'; print(json.dumps(d))" >> $OUT || return 1
  tail -1 $OUT | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['label'], d['echoes_per_s'], d.get('pass_timeline_us'))"
}
base_runs() {  # A/B on one box: the same device shapes with the build in $BASE (ws_loopback + its .so)
  run c1_split_base "GEVWS_LB_SPLIT=64" $BASE/ws_loopback --conns 100 --loops 1 --client-threads 2 --msg 128 || return 1
  run c1_one_base "GEVWS_LB_SPLIT=0" $BASE/ws_loopback --conns 100 --loops 1 --client-threads 2 --msg 128 || return 1
  run wss_8loops_base "X=1" $BASE/ws_loopback --conns 100 --loops 8 --client-threads 4 --mode wsserver || return 1
  if [ -n "$BASE_QUEUES" ]; then  # the base build with more hardware queues per process
    run wss_8loops_base_q$BASE_QUEUES "GPU_MAX_HW_QUEUES=$BASE_QUEUES" $BASE/ws_loopback --conns 100 --loops 8 \
      --client-threads 4 --mode wsserver || return 1
  fi
}
for i in 1 2; do
  if [ -n "$BASE" ] && [ -n "$BASE_FIRST" ]; then base_runs || exit 1; fi
  run c1_split "GEVWS_LB_SPLIT=64" gev_amd/ws_loopback --conns 100 --loops 1 --client-threads 2 --msg 128 || exit 1
  run c1_one "GEVWS_LB_SPLIT=0" gev_amd/ws_loopback --conns 100 --loops 1 --client-threads 2 --msg 128 || exit 1
  run c1_cpu "X=1" tools/ws_loopback_cpu --conns 100 --loops 1 --client-threads 2 --msg 128 || exit 1
  run wss_8loops "X=1" gev_amd/ws_loopback --conns 100 --loops 8 --client-threads 4 --mode wsserver || exit 1
  run wss_8loops_cpu "X=1" tools/ws_loopback_cpu --conns 100 --loops 8 --client-threads 4 --mode wsserver || exit 1
  if [ -n "$BASE" ] && [ -z "$BASE_FIRST" ]; then base_runs || exit 1; fi
done
