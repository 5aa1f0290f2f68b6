#!/bin/bash
# round 6: CG prologue partial loads issued together -- all GPU tests with the
# in-tree build, then default-bench and config-3 A/B against LIB_A
# usage: tools/ab/r6_prologue_ab.sh TAG LIB_A
set -u
TAG=$1; A=$2; B=optical-flow-python_amd/optical_flow/_lib/liboptflow.so
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
tools/gpu_step.sh 700 $O/gpu_tests.log python -u -m pytest -v -rA --timeout 300 --timeout-method thread tests -m gpu || exit $?
grep -q " passed" $O/gpu_tests.log && ! grep -q " failed" $O/gpu_tests.log || { echo "tests failed"; exit 1; }
for rep in 1 2; do for L in $A $B; do
  echo "== $L rep $rep" >> $O/bench_ab.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 200 $O/bench_tmp.log python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile --no-stream || exit $?
  grep '^{' $O/bench_tmp.log >> $O/bench_ab.log
done; done
for L in $A $B; do
  echo "== $L cfg3" >> $O/bench_ab.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 200 $O/bench_tmp.log python -u bench.py --method classic-c --solver pcg --height 720 --width 1280 --steps 4 --no-cpu-baseline --no-profile --no-stream || exit $?
  grep '^{' $O/bench_tmp.log >> $O/bench_ab.log
done
