# round 6: C2's unmask runs 1.20 x a same-size copy (C3's 0.985): every 4 KiB
# tile holds one whole frame at an unaligned source, so each takes v3's
# window path.  A/B against unmask variant 1 (v5's pipelined windows and
# chunk map for every batch), alternating, C2 and C5.  Predicted: if the
# window's dependent record loads are the cost, v5 -5 % on C2's unmask; if
# its extra LDS map work dominates, +5 % (then v3 stays).
set -o pipefail
cd $GRAFT_REPO_ROOT
JSONL=r06w_unmask_v5 bash scripts/gpu.sh 'bench r06w_c2_a --config c2' 'bench r06w_c2_v5a --config c2 --unmask-variant 1' \
  'bench r06w_c2_v5b --config c2 --unmask-variant 1' 'bench r06w_c2_b --config c2' \
  'bench r06w_c5_a --config c5' 'bench r06w_c5_v5a --config c5 --unmask-variant 1' \
  'bench r06w_c5_v5b --config c5 --unmask-variant 1' 'bench r06w_c5_b --config c5'
