#!/bin/bash
# round 3: fine-solve token with 2 slots and fewer, taller k_cgs bands (two
# fine solves side by side at half the chip each) vs the default (1 slot,
# 504 blocks); host-to-host bench, 2 reps; lanes 3 (default) and 4
set -e
: > gpurun_out/r3y_ab.log
for rep in 1 2; do
  for L in tools/ab/libbase2.so tools/ab/libs2b252.so tools/ab/libs2b336.so tools/ab/libs2b504.so; do
    echo "== $L rep $rep" >> gpurun_out/r3y_ab.log
    OPTFLOW_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile 2>/dev/null | grep '^{' >> gpurun_out/r3y_ab.log
  done
  for L in tools/ab/libbase2.so tools/ab/libs2b252.so; do
    echo "== $L lanes 4 rep $rep" >> gpurun_out/r3y_ab.log
    OPTFLOW_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --lanes 4 2>/dev/null | grep '^{' >> gpurun_out/r3y_ab.log
  done
done
