# A/B of gev_amd/ws_loopback against ab_base/ on the three live shapes.  Used
# once (profiles/r05/r05aa_queues_ab.jsonl) for a server build that called
# setenv("GPU_MAX_HW_QUEUES", "16") in main -- which the HIP runtime, loaded
# before main, ignored, so those runs are an A/A of two equal builds --
# beside the CPU twin; a warm-up run, then ROUNDS (default 4)
# alternating rounds whose order flips.  Lines -> gpurun_out/${TAG}_queues_ab.jsonl
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
export GEV_LOG_LEVEL=FATAL
OUT=gpurun_out/${TAG:-r05}_queues_ab.jsonl
WSS="--conns 100 --loops 8 --client-threads 4 --mode wsserver"
LB4K="--conns 4000 --loops 4 --client-threads 8 --msg 128"
C1="--conns 100 --loops 1 --client-threads 2 --msg 128"
run() {  # run <label> <binary> <args...>
  local label=$1 bin=$2; shift 2
  timeout -k 5 60 $bin --seconds 3 "$@" | grep '^{' | \
    python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['label']='$label'; print(json.dumps(d))" >> $OUT || return 1
  tail -1 $OUT | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); t=d.get('pass_timeline_us') or {}; print(d['label'], d['echoes_per_s'], t.get('launch'), t.get('wait'), t.get('gpu_decode'), t.get('gpu_gap'))"
}
run warmup gev_amd/ws_loopback $WSS || exit 1
for i in $(seq ${ROUNDS:-4}); do
  for shape in WSS LB4K C1; do
    args=${!shape}
    if [ $((i % 2)) = 1 ]; then
      run ${shape}_new gev_amd/ws_loopback $args || exit 1
      run ${shape}_base ab_base/ws_loopback $args || exit 1
    else
      run ${shape}_base ab_base/ws_loopback $args || exit 1
      run ${shape}_new gev_amd/ws_loopback $args || exit 1
    fi
    run ${shape}_cpu tools/ws_loopback_cpu $args || exit 1
  done
done
