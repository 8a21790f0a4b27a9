# round 6, final tree: the default bench line again (r06s's lacked its
# traffic field: profiles/ had been left out of the upload), then the three
# live shapes, 3 alternating rounds: this tree, the round's service commit
# (ab_base/: before the lazy last-call event) and the CPU twin.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh 'full r06t_default' && \
TAG=r06t ROUNDS=3 SHAPES="WSS LB4K C1" timeout -k 10 600 bash scripts/lb_ab.sh
