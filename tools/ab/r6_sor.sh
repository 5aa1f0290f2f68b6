#!/bin/bash
# round 6: SOR kernels -- every SOR test (bitwise vs the per-sweep kernel),
# then the config-2 bench line with OF_OPT_SOR_PIPELINE 1 and 2
# usage: tools/ab/r6_sor.sh TAG
set -u
TAG=$1
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
tools/gpu_step.sh 300 $O/sor_tests.log python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_stages.py -k "sor" || exit $?
grep -q " passed" $O/sor_tests.log && ! grep -q " failed" $O/sor_tests.log || { echo "tests failed"; exit 1; }
for m in 2 1; do
  tools/gpu_step.sh 300 $O/bench_cfg2_m$m.log python -u bench.py --method hs --solver sor --height 480 --width 640 --no-cpu-baseline --no-stream --sor-pipeline $m || exit $?
done
