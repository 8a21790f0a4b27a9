# round 6: the encode's box-dependent term (k_encode6 ÷
# the same process's unmask 1.02-1.10 across boxes, the unmask itself ~1 %).
# Request-size PMC passes + a kernel trace of the C4 encode with the same
# process's decode after it.  Predicted: if the term is bytes, the encode's
# read + write requests exceed its algorithmic L + (h' + L) by the 5-10 % it
# varies by (boundary chunks re-reading interior lines past L2); if they sit
# within ~1 % like the unmask's, the term is time per byte, not traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
CONFIGS=c4enc PREFIX=r06o PROG="tools/bench_encode.py --config c4 --rounds 1 --reps 3 --decode-reps 3" \
  bash scripts/gpu_pmc_split.sh
