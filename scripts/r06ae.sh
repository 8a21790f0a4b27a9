# round 6: C1 launched vs direct dispatch again, now that the one-launch
# kernel is 6.4 us (DPP scans; r06q/r06r measured direct level with a 8.6 us
# kernel: launch 3.6 -> 1.0 us but wait 0.3 -> 2.8 us).  Predicted: direct's
# wait back under 1 us, its launch + wait ~2.5 us under the launched pass's,
# echoes/s +1-3 % (inside C1's run spread, so read from the timeline).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=r06ae ROUNDS=3 SHAPES=C1 NO_SVC=1 DIRECT=1 timeout -k 10 400 bash scripts/lb_service_ab.sh
