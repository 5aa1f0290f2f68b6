#!/bin/bash
# config-3 bench A/B (Classic-C + 'pcg', 720p) of library builds, 2 reps each
# usage: tools/ab/cfg3_ab.sh TAG LIB...
set -u
TAG=$1; shift
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do for L in "$@"; do
  echo "== $L rep $rep" >> $O/bench_ab.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 300 $O/bench_tmp.log python -u bench.py --method classic-c --solver pcg \
      --height 720 --width 1280 --no-cpu-baseline --no-profile || exit $?
  grep '^{' $O/bench_tmp.log >> $O/bench_ab.log
done; done
