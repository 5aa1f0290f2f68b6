#!/bin/bash
# weighted-median A/B on the GPU box: WMF parity tests with the in-tree
# library, then per-launch time of each library build (1080p, 3 rounds,
# alternating) and the default bench (host to host, no profiling) per build.
# usage: tools/ab/wmf_ab.sh TAG LIB_A LIB_B
set -u
TAG=$1; A=$2; B=$3
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
tools/gpu_step.sh 300 $O/wmf_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_batch.py tests/test_gpu_stages.py tests/test_gpu_e2e.py -k "batch or pairs or slot or rccl or weighted_median or wmf or nl-fast or rubberwhale" || exit $?
grep -q " passed" $O/wmf_tests.log && ! grep -q " failed" $O/wmf_tests.log || { echo "WMF tests failed"; exit 1; }
for rep in 1 2 3; do for L in $A $B; do
  tools/gpu_step.sh 120 $O/wmf_bench_tmp.log python -u tools/wmf_bench.py --lib $L --reps 20 || exit $?
  cat $O/wmf_bench_tmp.log >> $O/wmf_bench.log
done; done
for rep in 1 2; do for L in $A $B; do
  echo "== $L rep $rep" >> $O/bench_ab.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 300 $O/bench_tmp.log python -u bench.py --steps 6 --no-cpu-baseline --no-profile || exit $?
  grep '^{' $O/bench_tmp.log >> $O/bench_ab.log
done; done
