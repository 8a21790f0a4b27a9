# round 6: r06m's lazy last-call event cut C1's launch phase 4.7-5.3 -> 3.4-3.7
# us but the wsserver shape (decode + chained handler step a pass, both lazy)
# fell 322-346 -> 235-267 k echoes/s, its launch phase 13-15 -> 21-24 us and
# its GPU decode 9.4 -> 11 us.  This build records the event after the
# handler step again (the decode alone stays lazy).  Predicted: if the loss
# comes from passes without a trailing marker, wsserver back to base
# (+-5 %) with C1's launch still ~3.6 us; if it comes from the decode and the
# handler launched back to back, wsserver stays ~25 % down (then: revert).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=r06n ROUNDS=3 SHAPES="WSS C1" timeout -k 10 400 bash scripts/lb_ab.sh
