# round 6: the wsserver shape measured 3-6 % below the round's service
# commit in r06u / r06ab but above it in r06n (the lazy-event build).  This
# runs the current tree against the r06n build itself (ab_base_lazy/, commit
# 3a56e59), wsserver only, 4 alternating rounds.  Predicted: if nothing after
# r06n touched the wsserver path, level (+-5 %); a consistent gap names the
# commits since (direct dispatch, ABI 3, DPP scans) as the place to look.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=r06ac BASE=ab_base_lazy ROUNDS=4 SHAPES="WSS" timeout -k 10 500 bash scripts/lb_ab.sh
