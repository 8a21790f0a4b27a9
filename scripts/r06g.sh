# round 6: the tests added after the mid-round suite (live-pass hypothesis
# property, split-walk re-walk count)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh 'test tests/test_gpu_properties.py::test_live_pass_decode_equals_oracle tests/test_gpu_split.py::test_split_walk_counts_its_serial_rewalks'
