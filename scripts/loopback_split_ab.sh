# Live-server A/B of split device passes (GEVWS_LB_SPLIT, GEVWS_LB_WAYS) against one pass per
# iteration and the CPU-decode twin, interleaved, two rounds; lines appended to
# gpurun_out/${TAG:-r04}_loopback_split.jsonl (split = the env value, 0 = off).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}; cd $R; mkdir -p gpurun_out
for i in 1 2; do
 for cfg in "--conns 100 --loops 1 --client-threads 2 --msg 128" "--conns 4000 --loops 4 --client-threads 8 --msg 128" "--conns 100 --loops 8 --client-threads 4 --mode wsserver"; do
  for v in 0 16:2 16:3 16:4 cpu; do
   b=gev_amd/ws_loopback; [ $v = cpu ] && b=tools/ws_loopback_cpu
   sp=${v%%:*}; w=${v##*:}; [ $v = cpu ] && sp=0 && w=1; [ $v = 0 ] && w=1
   GEVWS_LB_SPLIT=$sp GEVWS_LB_WAYS=$w timeout -k 5 60 $b --seconds 3 $cfg | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['bin']='$b'; d['cfg']='$cfg'; d['split']=$sp; d['ways']=$w; print(json.dumps(d))" >> gpurun_out/${TAG:-r04}_loopback_split.jsonl
  done
 done
done
