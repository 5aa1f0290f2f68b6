#!/bin/bash
# lanes sweep of the default bench (no profiled replay, no CPU baseline), 2 reps each
# usage: tools/ab/lanes_ab.sh TAG LANES...
set -u
TAG=$1; shift
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do for L in "$@"; do
  echo "== lanes $L rep $rep" >> $O/lanes_ab.log
  tools/gpu_step.sh 300 $O/bench_tmp.log python -u bench.py --steps 6 --lanes $L --no-cpu-baseline --no-profile || exit $?
  grep '^{' $O/bench_tmp.log >> $O/lanes_ab.log
done; done
