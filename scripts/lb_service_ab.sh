# A/B of the resident decode service on the live server: gev_amd/ws_loopback
# with launched passes (default) vs GEVWS_LB_SERVICE=1 (posted), beside the
# CPU twin, on the 100-connection shapes: a warm-up run, then ROUNDS rounds
# whose default / service order alternates.  One JSON line per run (label,
# then the loopback's line) -> gpurun_out/${TAG}_lb_service.jsonl
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
export GEV_LOG_LEVEL=FATAL
OUT=gpurun_out/${TAG:-r06}_lb_service.jsonl
WSS="--conns 100 --loops 8 --client-threads 4 --mode wsserver"
C1="--conns 100 --loops 1 --client-threads 2 --msg 128"
run() {  # run <label> <env> <binary> <args...>
  local label=$1 envv=$2 bin=$3; shift 3
  env $envv timeout -k 5 60 $bin --seconds ${SECONDS_PER_RUN:-3} "$@" | grep '^{' | \
    python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['label']='$label'; print(json.dumps(d))" >> $OUT || return 1
  tail -1 $OUT | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); t=d.get('pass_timeline_us') or {}; print(d['label'], d['echoes_per_s'], t.get('launch'), t.get('wait'), t.get('gpu_decode'), t.get('signalled_share'), t.get('service_share'), t.get('direct_share'))"
}
run warmup GEVWS_NOP=1 gev_amd/ws_loopback $C1 || exit 1
for i in $(seq ${ROUNDS:-3}); do
  for shape in ${SHAPES:-C1 WSS}; do
    args=${!shape}
    if [ $((i % 2)) = 1 ]; then
      run ${shape}_dev GEVWS_NOP=1 gev_amd/ws_loopback $args || exit 1
      [ "${NO_SVC:-0}" = 1 ] || run ${shape}_svc GEVWS_LB_SERVICE=1 gev_amd/ws_loopback $args || exit 1
    else
      [ "${NO_SVC:-0}" = 1 ] || run ${shape}_svc GEVWS_LB_SERVICE=1 gev_amd/ws_loopback $args || exit 1
      run ${shape}_dev GEVWS_NOP=1 gev_amd/ws_loopback $args || exit 1
    fi
    if [ "${DIRECT:-0}" = 1 ]; then  # the context's own AQL queue (gevws_ctx_set_direct)
      run ${shape}_direct GEVWS_LB_DIRECT=1 gev_amd/ws_loopback $args || exit 1
    fi
    run ${shape}_cpu GEVWS_NOP=1 tools/ws_loopback_cpu $args || exit 1
  done
done
