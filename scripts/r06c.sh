# round 6, third box: the 8-way C4 share's split walk with its serial
# re-walk count (rank 0 and rank 7), then the live shapes against the
# round-5 build (ab_base/) and the CPU twin
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh 'bench r06c_s8r0 --config c4 --emulate-shard 0/8' 'bench r06c_s8r7 --config c4 --emulate-shard 7/8' 'bench r06c_s4r0 --config c4 --emulate-shard 0/4' && \
TAG=r06c PRIO_ALL=1 ROUNDS=3 bash scripts/lb_ab.sh
