# round 6, final tree: kernel traces (rocprofv3 --kernel-trace --stats) of
# C2 / C4 / C5 and C4's 8-way share, so every config's profile in
# profiles/r06 is of the shipped kernels (r06b's were taken mid-round,
# before the split walk's writer wave and the one-launch refactor).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh 'prof r06y_c2 --config c2 --steps 10' 'prof r06y_c5 --config c5 --steps 10' \
  'prof r06y_c4 --config c4 --steps 3' 'prof r06y_c4s8 --config c4 --emulate-shard 0/8 --steps 5'
