#!/bin/bash
# round 6: config-3 profile (tools/ab/r6_c3prof.sh), then the SOR tests and a
# config-2 A/B of OF_OPT_SOR_PIPELINE 1 vs 2 (k_sor_wg on rings >= 8 sweeps)
set -u
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r6i; mkdir -p $O
tools/gpu_step.sh 300 $O/sor_tests.log python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_stages.py -k "sor" || exit $?
grep -q " passed" $O/sor_tests.log && ! grep -q " failed" $O/sor_tests.log || { echo "tests failed"; exit 1; }
for rep in 1 2; do for m in 1 2; do
  echo "== mode $m rep $rep" >> $O/cfg2_ab.log
  tools/gpu_step.sh 200 $O/bench_tmp.log python -u bench.py --method hs --solver sor --height 480 --width 640 --steps 4 --no-cpu-baseline --no-profile --no-stream --sor-pipeline $m || exit $?
  grep '^{' $O/bench_tmp.log >> $O/cfg2_ab.log
done; done
tools/ab/r6_c3prof.sh
