#!/bin/bash
# SQ counters of k_wmf and k_cgs on one serial 1080p pair, two passes of at
# most 8 SQ counters each (MI355X_MICROARCH.md: one block's limit per pass)
set -u
OUT=gpurun_out/pmc_sq2_${1:-x}
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --steps 1 --warmup 0 --pairs 1 --lanes 1 --no-cpu-baseline --no-profile --no-stream"
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex 'k_wmf|k_cgs' -f csv -d $OUT -o sq1 -- python3 $B > $OUT/sq1.log 2>&1 || { echo "pass 1 rc $?"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM --kernel-include-regex 'k_wmf|k_cgs' -f csv -d $OUT -o sq2 -- python3 $B > $OUT/sq2.log 2>&1 || { echo "pass 2 rc $?"; exit 1; }
