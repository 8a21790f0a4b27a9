# A/B of the hardware-queue spread on the wsserver shape (8 loops, one context
# each): gev_amd/ (contexts cycle their stream priority) vs ab_base/ (every
# context at the default priority), each with the runtime's default hardware
# queues and with GPU_MAX_HW_QUEUES=16, beside the CPU twin; alternating, three
# rounds.  Lines -> gpurun_out/${TAG}_wss_queues_ab.jsonl
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
export GEV_LOG_LEVEL=FATAL
OUT=gpurun_out/${TAG:-r05v}_wss_queues_ab.jsonl
run() {  # run <label> <env> <binary>
  env $2 timeout -k 5 60 $3 --seconds 3 --conns 100 --loops 8 --client-threads 4 --mode wsserver | grep '^{' | \
    python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['label']='$1'; d['env']='$2'; print(json.dumps(d))" >> $OUT || return 1
  tail -1 $OUT | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); t=d.get('pass_timeline_us') or {}; print(d['label'], d['echoes_per_s'], t.get('launch'), t.get('wait'), t.get('gpu_decode'), t.get('gpu_handler'), t.get('gpu_gap'))"
}
for i in 1 2 3; do
  run cycled "X=1" gev_amd/ws_loopback || exit 1
  run base "X=1" ab_base/ws_loopback || exit 1
  run cycled_q16 "GPU_MAX_HW_QUEUES=16" gev_amd/ws_loopback || exit 1
  run base_q16 "GPU_MAX_HW_QUEUES=16" ab_base/ws_loopback || exit 1
  run cpu "X=1" tools/ws_loopback_cpu || exit 1
done
