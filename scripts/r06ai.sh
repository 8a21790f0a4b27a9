# round 6, final tree: a soak of the live server -- each shape for 30 s with
# every echo checked byte for byte (errors must stay 0), and the opt-in forms
# (resident service, direct dispatch) for 20 s on C1; one JSON line each.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export GEV_LOG_LEVEL=FATAL
OUT=gpurun_out/r06ai_soak.jsonl
run() {  # label env seconds args...
  local label=$1 envv=$2 secs=$3; shift 3
  env $envv timeout -k 5 $((secs + 60)) gev_amd/ws_loopback --seconds $secs "$@" | grep '^{' | \
    python3 -c "import sys,json; d=json.loads(sys.stdin.read()); d['label']='$label'; print(json.dumps(d)); assert d['errors']==0, d['errors']" >> $OUT
}
run C1 GEVWS_NOP=1 30 --conns 100 --loops 1 --client-threads 2 --msg 128 &&
run LB4K GEVWS_NOP=1 30 --conns 4000 --loops 4 --client-threads 8 --msg 128 &&
run WSS GEVWS_NOP=1 30 --conns 100 --loops 8 --client-threads 4 --mode wsserver &&
run C1_64K GEVWS_NOP=1 20 --conns 16 --loops 1 --client-threads 2 --msg 65536 &&
run C1_service GEVWS_LB_SERVICE=1 20 --conns 100 --loops 1 --client-threads 2 --msg 128 &&
run C1_direct GEVWS_LB_DIRECT=1 20 --conns 100 --loops 1 --client-threads 2 --msg 128 &&
python3 -c "
import json
for l in open('$OUT'):
    d=json.loads(l); t=d.get('pass_timeline_us') or {}
    print(d['label'], d['echoes_per_s'], d['errors'], d.get('client_checked_echoes'), t.get('passes'), t.get('signalled_share'))
"
