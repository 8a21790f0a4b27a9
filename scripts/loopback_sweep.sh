set -e
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
for i in 1 2; do
 for b in gev_amd/ws_loopback tools/ws_loopback_cpu; do
  for cfg in "--conns 100 --loops 8 --client-threads 4 --mode wsserver" "--conns 100 --loops 1 --client-threads 2 --msg 128" "--conns 4000 --loops 4 --client-threads 8 --msg 128"; do
   timeout -k 5 60 $b --seconds 3 $cfg | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['bin']='$b'; d['cfg']='$cfg'; print(json.dumps(d))" >> gpurun_out/${TAG:-r04}_loopback.jsonl
  done
 done
done
