#!/bin/bash
# rocprofv3 passes for one bench configuration (run on the GPU box):
#   1. kernel trace + stats            (durations per dispatch)
#   2. PMC FETCH_SIZE                  (its own pass: MI355X_MICROARCH.md §rocprofv3)
#   3. PMC WRITE_SIZE                  (its own pass)
#   4. PMC TCC_HIT_sum TCC_MISS_sum    (L2 hit rate)
# usage: tools/profile.sh TAG [bench args...]
set -u
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile $*"
KRE='cg|wmf|flow_operator|partial_deriv|rof|minmax|update_occ|median|f2_to_planar'
tools/gpu_step.sh 300 $OUT/trace.log rocprofv3 --kernel-trace --stats -f csv -d $OUT -o trace -- python3 $B || exit $?
tools/gpu_step.sh 600 $OUT/fetch.log rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT -o fetch -- python3 $B || exit $?
tools/gpu_step.sh 600 $OUT/write.log rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT -o write -- python3 $B || exit $?
tools/gpu_step.sh 600 $OUT/l2.log rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KRE" -f csv -d $OUT -o l2 -- python3 $B || exit $?
