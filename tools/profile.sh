#!/bin/bash
# rocprofv3 passes for the bench (run on the GPU box):
#   1. kernel trace + stats of the default bench command (durations per dispatch),
#      and of bench.py --lanes 1 (the isolated durations the bench roofline uses)
#   2-4. PMC FETCH_SIZE / WRITE_SIZE / TCC hit+miss, each in its own pass
#        (MI355X_MICROARCH.md rocprofv3 section), on one serial 1080p pair
#   5. PMC SQ_INSTS_VALU / SQ_WAVES of the weighted median (its VALU-issue
#      roofline in the bench line)
# usage: tools/profile.sh TAG
set -u
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
S="bench.py --steps 1 --warmup 0 --pairs 1 --lanes 1 --no-cpu-baseline --no-profile"
KRE='k_cgs|k_cgp|k_wmf|k_flow_operator|k_partial_deriv|k_rof_iters|k_update_occ'
tools/gpu_step.sh 400 $OUT/trace.log rocprofv3 --kernel-trace --stats -f csv -d $OUT -o trace -- python3 bench.py || exit $?
# the isolated replay's counterpart (bench roofline = lanes 1 durations)
tools/gpu_step.sh 400 $OUT/trace1.log rocprofv3 --kernel-trace --stats -f csv -d $OUT -o trace1 -- python3 bench.py --lanes 1 --no-cpu-baseline --no-profile || exit $?
tools/gpu_step.sh 300 $OUT/fetch.log rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT -o fetch -- python3 $S || exit $?
tools/gpu_step.sh 300 $OUT/write.log rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT -o write -- python3 $S || exit $?
tools/gpu_step.sh 300 $OUT/l2.log rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KRE" -f csv -d $OUT -o l2 -- python3 $S || exit $?
tools/gpu_step.sh 300 $OUT/valu.log rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-include-regex 'k_wmf' -f csv -d $OUT -o valu -- python3 $S || exit $?
