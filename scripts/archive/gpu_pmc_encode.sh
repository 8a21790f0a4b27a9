#!/bin/bash
# SQ instruction-mix counters for the encode (and the decode it runs first), C4.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C=${CFG:-c4}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
  -d $OUT/pmc_enc_sq -o enc --output-format csv -- python3 $R/tools/bench_encode.py --config $C --reps 1 --rounds 1 > $OUT/pmc_enc_sq.log 2>&1
rc=$?; echo "sq rc=$rc"; tail -2 $OUT/pmc_enc_sq.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA \
  -d $OUT/pmc_enc_sq2 -o enc --output-format csv -- python3 $R/tools/bench_encode.py --config $C --reps 1 --rounds 1 > $OUT/pmc_enc_sq2.log 2>&1
rc=$?; echo "sq2 rc=$rc"; tail -2 $OUT/pmc_enc_sq2.log; exit $rc
