# A/B of one environment setting on the wsserver shape (8 loops, 100 clients):
# gev_amd/ws_loopback with and without $AB_ENV (e.g. GEVWS_LB_SPLIT=0: one
# decoder -- one context, one stream -- per loop instead of two), alternating,
# ROUNDS rounds (default 4) after a warm-up, beside the CPU twin.
# Lines -> gpurun_out/${TAG}_wss_env_ab.jsonl
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
export GEV_LOG_LEVEL=FATAL
OUT=gpurun_out/${TAG:-r05}_wss_env_ab.jsonl
WSS="--conns 100 --loops 8 --client-threads 4 --mode wsserver"
run() {  # run <label> <env> <binary>
  env $2 timeout -k 5 60 $3 --seconds 3 $WSS | grep '^{' | \
    python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['label']='$1'; d['env']='$2'; print(json.dumps(d))" >> $OUT || return 1
  tail -1 $OUT | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); t=d.get('pass_timeline_us') or {}; print(d['label'], d['echoes_per_s'], t.get('launch'), t.get('wait'), t.get('gpu_decode'), t.get('gpu_handler'), t.get('gpu_gap'))"
}
run warmup "X=1" gev_amd/ws_loopback || exit 1
for i in $(seq ${ROUNDS:-4}); do
  if [ $((i % 2)) = 1 ]; then
    run with "$AB_ENV" gev_amd/ws_loopback || exit 1
    run without "X=1" gev_amd/ws_loopback || exit 1
  else
    run without "X=1" gev_amd/ws_loopback || exit 1
    run with "$AB_ENV" gev_amd/ws_loopback || exit 1
  fi
  run cpu "X=1" tools/ws_loopback_cpu || exit 1
done
