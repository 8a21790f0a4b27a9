# round 6, final tree: the three live shapes, 3 alternating rounds against
# the round's service commit (ab_base/) and the CPU twin, for DESIGN §5.3's
# table (r06c's was taken before the lazy last-call event and the DPP scans).
# Predicted: C1 +2-5 % over ab_base (launch -1.5 us, kernel -2.2 us hidden),
# 4 000 / 4 and wsserver within their +-5-10 % spread.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=r06ag ROUNDS=3 SHAPES="C1 LB4K WSS" timeout -k 10 700 bash scripts/lb_ab.sh
