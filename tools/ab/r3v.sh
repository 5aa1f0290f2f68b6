#!/bin/bash
# round 3: k_cgs branch-free drain trim (OOB load offsets) and preprocessing without the lanes' token
set -u
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
: > gpurun_out/r3v_bitwise.log
for L in tools/ab/libbase.so tools/ab/libtrim2.so tools/ab/libtrim2pre0.so; do
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/ab/bitwise.py >> gpurun_out/r3v_bitwise.log 2>&1 || exit $?
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/ab/bitwise.py 864 1536 >> gpurun_out/r3v_bitwise.log 2>&1 || exit $?
done
bash tools/ab/bench_ab.sh tools/ab/libbase.so tools/ab/libtrim2.so tools/ab/libpretok0.so tools/ab/libtrim2pre0.so
