#!/bin/bash
# A/B of two library builds on the GPU box: parity tests (pytest args after
# the libraries) and smoke() with LIB_B, then the default bench (no profiled
# replay, no CPU baseline), alternating, 2 reps each.
# usage: tools/ab/lib_ab.sh TAG LIB_A LIB_B [pytest args...]
set -u
TAG=$1; A=$2; B=$3; shift 3
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
if [ $# -gt 0 ]; then
  OPTFLOW_LIB=$B tools/gpu_step.sh 600 $O/tests.log python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" || exit $?
  grep -q " passed" $O/tests.log && ! grep -q " failed" $O/tests.log || { echo "tests failed"; exit 1; }
fi
OPTFLOW_LIB=$B tools/gpu_step.sh 300 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
for rep in 1 2; do for L in $A $B; do
  echo "== $L rep $rep" >> $O/bench_ab.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 300 $O/bench_tmp.log python -u bench.py --steps 6 --no-cpu-baseline --no-profile || exit $?
  grep '^{' $O/bench_tmp.log >> $O/bench_ab.log
done; done
