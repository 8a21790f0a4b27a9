# round 6: where the writer-wave split walk pays -- the auto rule splits only
# batches of <= 32 connections per CU (the 8-way share).  Predicted: the 4-way
# share (64 per CU) split 8 ways -7 % (measured 2.607 -> 2.493 with the
# writer, unsplit 2.70), the 2-way share (128 per CU) split 4 ways -2 %, the
# full batch split 2 ways no gain (round 2: +11 % without the writer).
set -o pipefail
cd $GRAFT_REPO_ROOT
JSONL=r06i_split_rule bash scripts/gpu.sh 'bench r06i_s4_ks1 --config c4 --emulate-shard 0/4 --split-lanes 1' \
  'bench r06i_s4_ks8 --config c4 --emulate-shard 0/4 --split-lanes 8' 'bench r06i_s4_ks4 --config c4 --emulate-shard 0/4 --split-lanes 4' \
  'bench r06i_s4_ks16 --config c4 --emulate-shard 0/4 --split-lanes 16' \
  'bench r06i_s2_ks1 --config c4 --emulate-shard 0/2 --split-lanes 1' 'bench r06i_s2_ks4 --config c4 --emulate-shard 0/2 --split-lanes 4' \
  'bench r06i_s2_ks2 --config c4 --emulate-shard 0/2 --split-lanes 2' 'bench r06i_s2_ks8 --config c4 --emulate-shard 0/2 --split-lanes 8' \
  'bench r06i_c4_ks1 --config c4 --split-lanes 1' 'bench r06i_c4_ks2 --config c4 --split-lanes 2' \
  'bench r06i_s8_i2 --config c4 --emulate-shard 0/8 --inflight 2' 'bench r06i_s8 --config c4 --emulate-shard 0/8'
