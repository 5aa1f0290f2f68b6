#!/bin/bash
# round 6: config-2 A/B of two library builds (alternating, 2 reps each,
# no profiling replay), then B's mode-2 line
# usage: tools/ab/r6_sor_ab.sh TAG LIB_A LIB_B
set -u
TAG=$1; A=$2; B=$3
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do for L in $A $B; do
  echo "== $L rep $rep" >> $O/bench_ab.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 200 $O/bench_tmp.log python -u bench.py --method hs --solver sor --height 480 --width 640 --steps 4 --no-cpu-baseline --no-stream --no-profile || exit $?
  grep '^{' $O/bench_tmp.log >> $O/bench_ab.log
done; done
