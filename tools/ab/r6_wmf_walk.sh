#!/bin/bash
# round 6: weighted-median walk A/B -- every -m gpu test + smoke with the
# in-tree build, then per-launch time (3 reps) and the default bench (2 reps)
# alternating LIB_A and the in-tree build
# usage: tools/ab/r6_wmf_walk.sh TAG LIB_A
set -u
TAG=$1; A=$2; B=optical-flow-python_amd/optical_flow/_lib/liboptflow.so
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
tools/gpu_step.sh 700 $O/gpu_tests.log python -u -m pytest -v -s -rA --timeout 300 --timeout-method thread tests -m gpu || exit $?
tools/gpu_step.sh 150 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
for rep in 1 2 3; do for L in $A $B; do
  tools/gpu_step.sh 120 $O/wmf_tmp.log python -u tools/wmf_bench.py --lib $L --reps 20 || exit $?
  grep '^{' $O/wmf_tmp.log >> $O/wmf_bench.log
done; done
for rep in 1 2; do for L in $A $B; do
  echo "== $L rep $rep" >> $O/bench_ab.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 200 $O/bench_tmp.log python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile --no-stream || exit $?
  grep '^{' $O/bench_tmp.log >> $O/bench_ab.log
done; done
