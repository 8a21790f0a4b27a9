# round 6, second (last) full GPU suite, on the tree with the resident
# service, the lazy last-call event and direct dispatch; then on the same box
# smoke(), the default bench line (GPU + CPU legs) and the C3 bench under
# rocprofv3 --kernel-trace --stats (the profile the bench line's roofline
# cites).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh 'test -m gpu tests/' 'py tools/run_smoke.py' 'full r06s_default' 'prof r06s_c3 --steps 5 --warmup 2'
