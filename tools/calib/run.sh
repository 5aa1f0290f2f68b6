#!/bin/bash
# PMC calibration passes for tools/calib/calib_fetch (run on the GPU box)
set -u
OUT=gpurun_out/calib
mkdir -p $OUT
export TMPDIR=/tmp
tools/gpu_step.sh 120 $OUT/trace.log rocprofv3 --kernel-trace --stats -f csv -d $OUT -o trace -- tools/calib/calib_fetch || exit $?
tools/gpu_step.sh 120 $OUT/fetch.log rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT -o fetch -- tools/calib/calib_fetch || exit $?
tools/gpu_step.sh 120 $OUT/write.log rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT -o write -- tools/calib/calib_fetch || exit $?
