#!/bin/bash
# k_cgs variant A/B: isolated fixed-iteration CG timing (tools/pcg_bench.py,
# 1080p) and the default bench (timed lanes) per library, alternating, 2 reps
# usage: tools/ab/cgs_ab.sh TAG LIB...
set -u
TAG=$1; shift
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do for L in "$@"; do
  echo "== $L rep $rep" >> $O/pcg.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 120 $O/tmp.log python -u tools/pcg_bench.py --iters 200 || exit $?
  cat $O/tmp.log >> $O/pcg.log
done; done
for rep in 1 2; do for L in "$@"; do
  echo "== $L rep $rep" >> $O/bench_ab.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 300 $O/tmp.log python -u bench.py --steps 10 --no-cpu-baseline --no-profile || exit $?
  grep '^{' $O/tmp.log >> $O/bench_ab.log
done; done
