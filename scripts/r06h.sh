# round 6: the split walk with its entries through a writer wave (k_walk_split
# ST 2).  Written prediction: the 8-way share's walk 0.42 ->
# ~0.33 ms, its step 1.467 -> ~1.38 ms (-6 %), as the writer wave took the
# full C4 walk 1.60 -> 1.26 ms in round 3.  Parity first (split tests, the
# hypothesis split property, every walk variant), then alternating rounds of
# the new default against walk variant 4 (entries from the walking lanes).
set -o pipefail
cd $GRAFT_REPO_ROOT
P=tests/test_gpu_parity.py
bash scripts/gpu.sh "test $P::test_walk_variants_uniform_runs $P::test_escaped_entry_lengths $P::test_record_pass_groups" && \
JSONL=r06h_splitw bash scripts/gpu.sh 'bench r06h_new1 --config c4 --emulate-shard 0/8' 'bench r06h_old1 --config c4 --emulate-shard 0/8 --walk-variant 4' \
  'bench r06h_old2 --config c4 --emulate-shard 0/8 --walk-variant 4' 'bench r06h_new2 --config c4 --emulate-shard 0/8' \
  'bench r06h_new7 --config c4 --emulate-shard 7/8' 'bench r06h_old7 --config c4 --emulate-shard 7/8 --walk-variant 4' \
  'bench r06h_new4 --config c4 --emulate-shard 0/4 --split-lanes 8' 'bench r06h_old4 --config c4 --emulate-shard 0/4 --split-lanes 8 --walk-variant 4'
