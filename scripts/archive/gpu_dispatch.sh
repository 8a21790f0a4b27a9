#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.err; tail -c 1200 $OUT/$name.log; return $rc; }


run srv_c3 600 python tools/bench_server.py --config c3 --reps 5 || exit $?
export GEV_DIST_BACKEND=gloo
run bench_2rank 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config c2 --steps 20 --warmup 3 || exit $?
