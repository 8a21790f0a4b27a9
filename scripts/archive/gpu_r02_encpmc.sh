#!/bin/bash
# SQ counter passes (separate runs) over tools/bench_encode.py on C4: the
# encode kernel beside the decode's unmask kernel of the same batch.
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $R
V=${ENC_V:-0}
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $CTRS -d $OUT/encpmc_$i -o p --output-format csv -- \
    python tools/bench_encode.py --config ${CFG:-c4} --variants $V --rounds 1 --reps 2 > $OUT/encpmc_$i.log 2>&1 || { tail -5 $OUT/encpmc_$i.log; exit 1; }
done
echo done
