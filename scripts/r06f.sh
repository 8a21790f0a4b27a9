# round 6, mid-round: the full GPU suite once (budget: two per round), then
# on one box the default bench line (GPU + the CPU legs), the host-inclusive
# rate (pinned host -> H2D -> decode -> D2H, 64 MiB chunks x 2 streams and
# 32 MiB x 2), and the full C4 batch beside its 2- / 8-way shares
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh 'test -m gpu tests/' 'full r06f_default' \
  'py tools/host_inclusive.py --sweep 64:2,32:2,128:3 ' \
  'bench r06f_c4 --config c4' 'bench r06f_s2r0 --config c4 --emulate-shard 0/2' 'bench r06f_s8r0 --config c4 --emulate-shard 0/8' \
  'bench r06f_s8r0_i2 --config c4 --emulate-shard 0/8 --inflight 2'
