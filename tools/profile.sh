#!/bin/bash
# rocprofv3 passes for the bench (run on the GPU box):
#   1. kernel trace + stats of the bench command (durations per dispatch),
#      and of the same with --lanes 1 (the isolated durations the bench
#      roofline uses)
#   2-4. PMC FETCH_SIZE / WRITE_SIZE / TCC hit+miss, each in its own pass
#        (MI355X_MICROARCH.md rocprofv3 section), on one serial pair
#   5. PMC SQ_INSTS_VALU / SQ_WAVES of the weighted median (its VALU-issue
#      roofline in the bench line)
# usage: tools/profile.sh TAG [bench args for another config, e.g.
#        --method classic-c --solver pcg --height 720 --width 1280]
# then:  python tools/prof_summary.py gpurun_out/prof_TAG --H .. --W .. --traffic \
#        --workload method@HxW/solver
set -u
TAG=$1; shift
EXTRA="$*"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
S="bench.py $EXTRA --steps 1 --warmup 0 --pairs 1 --lanes 1 --no-cpu-baseline --no-profile --no-stream"
KRE='k_cgs|k_cgp|k_cg<|k_wmf|k_flow_operator|k_warp_operator|k_partial_deriv|k_rof_iters|k_update_occ|k_sor_pipe'
tools/gpu_step.sh 400 $OUT/trace.log rocprofv3 --kernel-trace --stats -f csv -d $OUT -o trace -- python3 bench.py $EXTRA --no-cpu-baseline || exit $?
tools/gpu_step.sh 400 $OUT/trace1.log rocprofv3 --kernel-trace --stats -f csv -d $OUT -o trace1 -- python3 bench.py $EXTRA --lanes 1 --no-cpu-baseline --no-profile --no-stream || exit $?
tools/gpu_step.sh 300 $OUT/fetch.log rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT -o fetch -- python3 $S || exit $?
tools/gpu_step.sh 300 $OUT/write.log rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT -o write -- python3 $S || exit $?
tools/gpu_step.sh 300 $OUT/l2.log rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KRE" -f csv -d $OUT -o l2 -- python3 $S || exit $?
tools/gpu_step.sh 300 $OUT/valu.log rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-include-regex 'k_wmf' -f csv -d $OUT -o valu -- python3 $S || exit $?
