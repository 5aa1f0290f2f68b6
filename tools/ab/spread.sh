#!/bin/bash
# run-to-run spread of the default bench's timed rates on one box: REPS runs
# (no profiled replay, no CPU baseline)
# usage: tools/ab/spread.sh TAG [REPS]
set -u
TAG=$1; REPS=${2:-5}
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
for rep in $(seq 1 $REPS); do
  tools/gpu_step.sh 300 $O/bench_tmp.log python -u bench.py --no-cpu-baseline --no-profile || exit $?
  grep '^{' $O/bench_tmp.log >> $O/spread.log
done
