#!/bin/bash
# round 3: WMF fp32 chunk sums (native ds_add_f32) and fine-solve block counts
set -u
export PYTHONDONTWRITEBYTECODE=1
: > gpurun_out/r3ac_wmf.log
for L in tools/ab/libdef.so tools/ab/libwmf32.so; do
  echo "== $L" >> gpurun_out/r3ac_wmf.log
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/wmf_bench.py >> gpurun_out/r3ac_wmf.log 2>&1 || exit $?
done
OPTFLOW_LIB=tools/ab/libwmf32.so timeout -k 10 200 python -u -m pytest -s -q --timeout 150 --timeout-method thread \
  tests/test_gpu_stages.py -m gpu -k "weighted_median" >> gpurun_out/r3ac_wmf.log 2>&1
echo "pytest rc $?" >> gpurun_out/r3ac_wmf.log
: > gpurun_out/r3ac_ab.log
for rep in 1 2; do
  for L in tools/ab/libdef.so tools/ab/libwmf32.so tools/ab/liblb224.so tools/ab/liblb288.so; do
    echo "== $L rep $rep" >> gpurun_out/r3ac_ab.log
    OPTFLOW_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile 2>/dev/null | grep '^{' >> gpurun_out/r3ac_ab.log || exit $?
  done
done
