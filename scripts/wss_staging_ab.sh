# A/B of the one-launch decode's staging slices on the wsserver shape: gev_amd/ (slices) vs
# ab_base/ (a build with one staging workgroup), alternating, four rounds.
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
export GEV_LOG_LEVEL=FATAL
for i in 1 2 3 4; do
  for b in gev_amd ab_base; do
    timeout -k 5 60 $b/ws_loopback --seconds 3 --conns 100 --loops 8 --client-threads 4 --mode wsserver | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['label']='wss_$b'; print(json.dumps(d))" >> gpurun_out/r05s_wss_ab.jsonl || exit 1
    tail -1 gpurun_out/r05s_wss_ab.jsonl | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); t=d.get('pass_timeline_us') or {}; print(d['label'], d['echoes_per_s'], t.get('launch'), t.get('wait'), t.get('gpu_decode'), t.get('gpu_handler'))"
  done
done
