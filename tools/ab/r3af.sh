#!/bin/bash
# round 3: k_cgs blocks of the 864x1536 fine solves in lanes mode (1080p stays 252)
set -e
: > gpurun_out/r3af_ab.log
for rep in 1 2; do
  for L in tools/ab/libd.so tools/ab/libs168.so tools/ab/libs196.so tools/ab/libs336.so; do
    echo "== $L rep $rep" >> gpurun_out/r3af_ab.log
    OPTFLOW_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile 2>/dev/null | grep '^{' >> gpurun_out/r3af_ab.log
  done
done
