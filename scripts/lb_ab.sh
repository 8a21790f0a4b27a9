# A/B of gev_amd/ws_loopback against ab_base/ (a previous round's build) and
# the CPU twin on the three live shapes: a warm-up run, then ROUNDS (default
# 3) rounds whose new / base order alternates; with PRIO_ALL=1 the new build's
# wsserver shape also runs with GEVWS_STREAM_PRIORITIES=all.  One JSON line
# per run (label, then the loopback's line) -> gpurun_out/${TAG}_lb_ab.jsonl
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
export GEV_LOG_LEVEL=FATAL
OUT=gpurun_out/${TAG:-r06}_lb_ab.jsonl
WSS="--conns 100 --loops 8 --client-threads 4 --mode wsserver"
LB4K="--conns 4000 --loops 4 --client-threads 8 --msg 128"
C1="--conns 100 --loops 1 --client-threads 2 --msg 128"
run() {  # run <label> <env> <binary> <args...>
  local label=$1 envv=$2 bin=$3; shift 3
  env $envv timeout -k 5 60 $bin --seconds ${SECONDS_PER_RUN:-3} "$@" | grep '^{' | \
    python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['label']='$label'; print(json.dumps(d))" >> $OUT || return 1
  tail -1 $OUT | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); t=d.get('pass_timeline_us') or {}; print(d['label'], d['echoes_per_s'], t.get('launch'), t.get('wait'), t.get('gpu_decode'), t.get('signalled_share'))"
}
run warmup GEVWS_NOP=1 gev_amd/ws_loopback $WSS || exit 1
for i in $(seq ${ROUNDS:-3}); do
  for shape in ${SHAPES:-WSS LB4K C1}; do
    args=${!shape}
    if [ $((i % 2)) = 1 ]; then
      run ${shape}_new GEVWS_NOP=1 gev_amd/ws_loopback $args || exit 1
      run ${shape}_base GEVWS_NOP=1 ${BASE:-ab_base}/ws_loopback $args || exit 1
    else
      run ${shape}_base GEVWS_NOP=1 ${BASE:-ab_base}/ws_loopback $args || exit 1
      run ${shape}_new GEVWS_NOP=1 gev_amd/ws_loopback $args || exit 1
    fi
    if [ "$shape" = WSS ] && [ "${PRIO_ALL:-0}" = 1 ]; then
      run ${shape}_new_all GEVWS_STREAM_PRIORITIES=all gev_amd/ws_loopback $args || exit 1
    fi
    run ${shape}_cpu GEVWS_NOP=1 tools/ws_loopback_cpu $args || exit 1
  done
done
