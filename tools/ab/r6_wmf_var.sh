#!/bin/bash
# round 6: weighted-median variant A/B -- WMF parity tests and smoke with the
# variant, per-launch time alternating (3 reps), default bench alternating
# usage: tools/ab/r6_wmf_var.sh TAG LIB_B
set -u
TAG=$1; B=$2; A=optical-flow-python_amd/optical_flow/_lib/liboptflow.so
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
OPTFLOW_LIB=$B tools/gpu_step.sh 400 $O/tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_stages.py tests/test_gpu_e2e.py tests/test_gpu_fullsize.py -k "(weighted_median or e2e or nl_fast or nl-fast or 1080) and not sor" || exit $?
grep -q " passed" $O/tests.log && ! grep -q " failed" $O/tests.log || { echo "tests failed"; exit 1; }
OPTFLOW_LIB=$B tools/gpu_step.sh 150 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
for rep in 1 2 3; do for L in $A $B; do
  tools/gpu_step.sh 120 $O/wmf_tmp.log python -u tools/wmf_bench.py --lib $L --reps 20 || exit $?
  grep '^{' $O/wmf_tmp.log >> $O/wmf_bench.log
done; done
for rep in 1 2; do for L in $A $B; do
  echo "== $L rep $rep" >> $O/bench_ab.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 200 $O/bench_tmp.log python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile --no-stream || exit $?
  grep '^{' $O/bench_tmp.log >> $O/bench_ab.log
done; done
