# round 6: the unsplit walk's writer wave below 128 chains per CU (walk
# variant 3 forces it).  Predicted: C5's walk (256 chains of ~163 hops, one
# chain per CU) 0.079 -> ~0.065 ms (-3 % of its step) as the split walk's
# went -13 % with it; C2 / C3 (16 chains per CU, speculation) within +-2 %.
set -o pipefail
cd $GRAFT_REPO_ROOT
JSONL=r06j_walk_writer bash scripts/gpu.sh 'bench r06j_c5_w0a --config c5' 'bench r06j_c5_w3a --config c5 --walk-variant 3' \
  'bench r06j_c5_w3b --config c5 --walk-variant 3' 'bench r06j_c5_w0b --config c5' \
  'bench r06j_c2_w0a --config c2' 'bench r06j_c2_w3a --config c2 --walk-variant 3' \
  'bench r06j_c2_w3b --config c2 --walk-variant 3' 'bench r06j_c2_w0b --config c2' \
  'bench r06j_c3_w0 --config c3 --steps 5' 'bench r06j_c3_w3 --config c3 --steps 5 --walk-variant 3'
