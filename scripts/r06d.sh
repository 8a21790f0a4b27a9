# round 6: the 8-way C4 share's header walk against its lanes per connection
# (GEVWS_TUNE_SPLIT_LANES 1 = unsplit .. 32), rank 0's share, to place the
# walk on a latency or a throughput floor
set -o pipefail
cd $GRAFT_REPO_ROOT
JSONL=r06d_split bash scripts/gpu.sh 'bench r06d_ks1 --config c4 --emulate-shard 0/8 --split-lanes 1' 'bench r06d_ks4 --config c4 --emulate-shard 0/8 --split-lanes 4' 'bench r06d_ks8 --config c4 --emulate-shard 0/8 --split-lanes 8' 'bench r06d_ks16 --config c4 --emulate-shard 0/8 --split-lanes 16' 'bench r06d_ks32 --config c4 --emulate-shard 0/8 --split-lanes 32' 'bench r06d_ks2 --config c4 --emulate-shard 0/8 --split-lanes 2'
