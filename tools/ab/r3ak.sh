#!/bin/bash
# round 3: 270 blocks (15 bands at 1080p) and 3 token slots, vs the default
set -e
: > gpurun_out/r3ak_ab.log
for rep in 1 2; do
  for L in tools/ab/libd.so tools/ab/libb270.so tools/ab/libs3.so; do
    echo "== $L rep $rep" >> gpurun_out/r3ak_ab.log
    OPTFLOW_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile 2>/dev/null | grep '^{' >> gpurun_out/r3ak_ab.log
  done
done
