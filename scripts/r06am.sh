# round 6, final build: the default bench line (the contract command: C3 with
# the CPU legs and the copy ceilings) and its kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh 'full r06am_default' 'prof r06am_c3 --steps 5 --warmup 2'
