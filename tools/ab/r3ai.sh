#!/bin/bash
# round 3: fine solves of the lanes on a high-priority stream (OF_SOLVE_PRIO)
set -e
: > gpurun_out/r3ai_ab.log
for rep in 1 2 3; do
  for L in tools/ab/libd.so tools/ab/libprio.so; do
    echo "== $L rep $rep" >> gpurun_out/r3ai_ab.log
    OPTFLOW_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile 2>/dev/null | grep '^{' >> gpurun_out/r3ai_ab.log
  done
done
