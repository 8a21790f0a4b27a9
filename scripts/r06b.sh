# round 6, second box: request-size PMC splits + kernel traces for C2 / C5
#  and C3 / C4 re-taken on this round's kernels, then the
# default bench line (CPU legs with the fresh / cache-hot allocation modes)
# and C5 / C2 against a size-matched copy in the same clock state
set -o pipefail
cd $GRAFT_REPO_ROOT
CONFIGS="c2 c5 c4 c3" PREFIX=r06b_split bash scripts/gpu_pmc_split.sh && \
bash scripts/gpu.sh 'full r06b_default' 'bench r06b_c5i --config c5 --copy-interleave 5' 'bench r06b_c2i --config c2 --copy-interleave 5'
