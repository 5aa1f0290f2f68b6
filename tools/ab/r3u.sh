#!/bin/bash
# round 3: bitwise + bench A/B of k_cgs drain trimming and the preprocessing token
set -u
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
: > gpurun_out/r3u_bitwise.log
for L in tools/ab/libbase.so tools/ab/libtrim.so tools/ab/libpretok0.so; do
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/ab/bitwise.py >> gpurun_out/r3u_bitwise.log 2>&1 || exit $?
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/ab/bitwise.py 540 960 >> gpurun_out/r3u_bitwise.log 2>&1 || exit $?
done
bash tools/ab/bench_ab.sh tools/ab/libbase.so tools/ab/libtrim.so tools/ab/libpretok0.so
