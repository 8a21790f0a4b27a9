# round 6: the record pass's segmented wave scan (wave_seg_scan, 64 frames a
# round) as a DPP inclusive scan minus the value before the lane's segment
# (one ballot + one shuffle) instead of a shuffled value and head flag at
# each of six steps (18 ds_bpermute round trips a round).  Parity first
# (decode / split / property tests: every walk and record-pass form), then
# C4 and its 8-way share alternating with the previous commit's library
# (ab_base_scan/, swapped in on the box).  Predicted: C4's record pass 0.48
# -> ~0.40 ms if the shuffles bound it, else unchanged (then reverted).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_split.py tests/test_gpu_properties.py > gpurun_out/r06ad_pytest.log 2>&1 &&
cp gev_amd/libgevws.so /tmp/libgevws.new.so &&
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cp ab_base_scan/libgevws.so gev_amd/libgevws.so; else cp /tmp/libgevws.new.so gev_amd/libgevws.so; fi
    JSONL=r06ad_emit bash scripts/gpu.sh "bench r06ad_c4_${v}$r --config c4 --steps 10" \
      "bench r06ad_s8_${v}$r --config c4 --emulate-shard 0/8 --steps 10" || exit 1
  done
done
cp /tmp/libgevws.new.so gev_amd/libgevws.so
