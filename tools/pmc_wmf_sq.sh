#!/bin/bash
# SQ counters of the weighted median on one serial 1080p pair (one pass):
# VALU / LDS / SALU instruction counts, wave cycles and LDS issue stalls
set -u
OUT=gpurun_out/pmc_wmf_sq_${1:-x}
mkdir -p $OUT
export TMPDIR=/tmp
tools/gpu_step.sh 300 $OUT/sq.log rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex 'k_wmf|k_cgs' -f csv -d $OUT -o sq -- python3 bench.py --steps 1 --warmup 0 --pairs 1 --lanes 1 --no-cpu-baseline --no-profile
