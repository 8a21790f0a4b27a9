#!/bin/bash
# Multi-rank rehearsal on ONE GPU (gloo; RCCL allows one rank per device): the
# torch.distributed.run launch the driver uses, 2 ranks sharing the card --
# C2 weak scaling and C4 strong scaling (LPT shard of one global batch).
# Timings are meaningless (two ranks share one GPU); this checks the N > 1
# code path end to end: launch, per-rank batches, verification, count
# all-reduce, max-over-ranks timing, rank-0 JSON line.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
run() { local name=$1 to=$2; shift 2; echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2> $OUT/$name.err; local rc=$?
  echo "$name rc=$rc"; tail -3 $OUT/$name.err; tail -c 900 $OUT/$name.log; echo; return $rc; }
export GEV_DIST_BACKEND=gloo
run rehearse_c2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config c2 --steps 10 --warmup 2 || exit $?
run rehearse_c4 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config c4 --steps 5 --warmup 1 || exit $?
