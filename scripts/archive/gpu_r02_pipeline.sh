#!/bin/bash
# Round 2: host-ingress pipelining -- the protocol tests (begin/end), the
# loopback tests, then the C1 loopback with the pipelined loop
# (GEVWS_LB_PIPELINE=1) vs the serial loop (default) vs the CPU decode, interleaved.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_loopback.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $OUT/pytest_pipe.log 2>&1
rc=$?; tail -3 $OUT/pytest_pipe.log; [ $rc -eq 0 ] || exit $rc
export GEV_LOG_LEVEL=FATAL
: > $OUT/loopback_pipeline_ab.jsonl
run() { local name=$1; shift; timeout -k 10 60 "$@" > $OUT/$name.log 2> $OUT/$name.err || { tail -3 $OUT/$name.err; exit 1; }
  python -c "
import json; d=json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1]); d['run']='$name'
print(json.dumps({k: d[k] for k in ('run','connections','loops','echoes_per_s','decode_us_per_pass','mean_conns_per_pass','errors')}))
open('$OUT/loopback_pipeline_ab.jsonl','a').write(json.dumps(d)+'\n')"; }
for rnd in 1 2; do
  GEVWS_LB_PIPELINE=1 run pipe_100_$rnd gev_amd/ws_loopback --conns 100 --loops 1 --msg 128 --seconds 3 --client-threads 2
  run serial_100_$rnd gev_amd/ws_loopback --conns 100 --loops 1 --msg 128 --seconds 3 --client-threads 2
  run cpu_100_$rnd tools/ws_loopback_cpu --conns 100 --loops 1 --msg 128 --seconds 3 --client-threads 2
done
GEVWS_LB_PIPELINE=1 run pipe_4000 gev_amd/ws_loopback --conns 4000 --loops 4 --msg 128 --seconds 3 --client-threads 8
run serial_4000 gev_amd/ws_loopback --conns 4000 --loops 4 --msg 128 --seconds 3 --client-threads 8
run cpu_4000 tools/ws_loopback_cpu --conns 4000 --loops 4 --msg 128 --seconds 3 --client-threads 8
