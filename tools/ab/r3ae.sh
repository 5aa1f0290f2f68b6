#!/bin/bash
# round 3: k_cgs halo lanes 4 (default) vs 5 (the degree-5 rho-recurrence terms
# reach 10 px from an output pixel); bench 2 reps + the full-size parity tests on h5
set -u
export PYTHONDONTWRITEBYTECODE=1
: > gpurun_out/r3ae_ab.log
for rep in 1 2; do
  for L in tools/ab/libh4.so tools/ab/libh5.so; do
    echo "== $L rep $rep" >> gpurun_out/r3ae_ab.log
    OPTFLOW_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile 2>/dev/null | grep '^{' >> gpurun_out/r3ae_ab.log || exit $?
  done
done
OPTFLOW_LIB=tools/ab/libh5.so timeout -k 10 400 python -u -m pytest -s -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fullsize.py tests/test_gpu_stages.py -m gpu > gpurun_out/r3ae_h5_tests.log 2>&1
echo "pytest rc $?" >> gpurun_out/r3ae_h5_tests.log
