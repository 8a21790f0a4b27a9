# A/B of the context stream-priority cycling on the 4 000-connection / 4-loop
# shape: gev_amd/ (cycled) vs ab_base/ (one priority), beside the CPU twin;
# a warm-up run, then alternating rounds (ROUNDS, default 3; the order flips each round).  Lines -> gpurun_out/${TAG}_lb4k_queues_ab.jsonl
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
export GEV_LOG_LEVEL=FATAL
OUT=gpurun_out/${TAG:-r05x}_lb4k_queues_ab.jsonl
run() {  # run <label> <binary> [env]
  env ${3:-X=1} timeout -k 5 60 $2 --seconds 3 --conns 4000 --loops 4 --client-threads 8 --msg 128 | grep '^{' | \
    python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['label']='$1'; print(json.dumps(d))" >> $OUT || return 1
  tail -1 $OUT | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); t=d.get('pass_timeline_us') or {}; print(d['label'], d['echoes_per_s'], t.get('launch'), t.get('wait'), t.get('gpu_decode'))"
}
run warmup gev_amd/ws_loopback || exit 1
for i in $(seq ${ROUNDS:-3}); do
  if [ $((i % 2)) = 1 ]; then
    run cycled gev_amd/ws_loopback || exit 1
    run base ab_base/ws_loopback || exit 1
    run base_q16 ab_base/ws_loopback GPU_MAX_HW_QUEUES=16 || exit 1
  else
    run base_q16 ab_base/ws_loopback GPU_MAX_HW_QUEUES=16 || exit 1
    run base ab_base/ws_loopback || exit 1
    run cycled gev_amd/ws_loopback || exit 1
  fi
  run cpu tools/ws_loopback_cpu || exit 1
done
