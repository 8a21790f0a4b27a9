# The live-server sweep: device (gev_amd/ws_loopback) against the CPU-decode
# twin (tools/ws_loopback_cpu) on the three shapes, ${RUNS:-2} runs each,
# one JSON line per run into gpurun_out/${TAG}_loopback.jsonl.  With
# PRIO_ALL=1 the device's wsserver shape also runs with
# GEVWS_STREAM_PRIORITIES=all (stream priorities above normal allowed).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
run() {  # bin cfg env
  env $3 timeout -k 5 60 $1 --seconds 3 $2 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['bin']='$1'; d['cfg']='$2'; d['env']='$3'; print(json.dumps(d))" >> gpurun_out/${TAG:-r06}_loopback.jsonl
}
for i in $(seq ${RUNS:-2}); do
 for b in gev_amd/ws_loopback tools/ws_loopback_cpu; do
  for cfg in "--conns 100 --loops 8 --client-threads 4 --mode wsserver" "--conns 100 --loops 1 --client-threads 2 --msg 128" "--conns 4000 --loops 4 --client-threads 8 --msg 128"; do
   run $b "$cfg" "GEVWS_NOP=1"
  done
 done
 if [ "${PRIO_ALL:-0}" = 1 ]; then
  run gev_amd/ws_loopback "--conns 100 --loops 8 --client-threads 4 --mode wsserver" "GEVWS_STREAM_PRIORITIES=all"
 fi
done
