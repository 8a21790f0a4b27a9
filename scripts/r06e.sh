# round 6: what bounds the 8-way C4 share's split walk -- SQ wave / wait /
# instruction counters and L1/L2 request counters for the walk at 16 lanes
# per connection and unsplit, and the full C4 walk beside them
set -o pipefail
cd $GRAFT_REPO_ROOT
SQ=SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_INSTS_VMEM_RD,SQ_INSTS_VALU,SQ_INSTS_LDS
MEM=TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum,TCP_TOTAL_CACHE_ACCESSES_sum,TCP_TCC_READ_REQ_sum,GRBM_GUI_ACTIVE
bash scripts/gpu.sh "pmc s8ks16_sq $SQ -- --config c4 --emulate-shard 0/8 --split-lanes 16 --steps 3 --warmup 1" \
  "pmc s8ks16_mem $MEM -- --config c4 --emulate-shard 0/8 --split-lanes 16 --steps 3 --warmup 1" \
  "pmc s8ks1_sq $SQ -- --config c4 --emulate-shard 0/8 --split-lanes 1 --steps 3 --warmup 1" \
  "pmc s8ks1_mem $MEM -- --config c4 --emulate-shard 0/8 --split-lanes 1 --steps 3 --warmup 1" \
  "pmc c4_sq $SQ -- --config c4 --steps 3 --warmup 1" \
  "pmc c4_mem $MEM -- --config c4 --steps 3 --warmup 1"
