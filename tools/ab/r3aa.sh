#!/bin/bash
# round 3: k_cgs blocks of the coarse (non-token) solves in lanes mode
set -e
: > gpurun_out/r3aa_ab.log
run() {  # lib lanes
  echo "== $1 lanes $2 rep $rep" >> gpurun_out/r3aa_ab.log
  OPTFLOW_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --lanes $2 2>/dev/null | grep '^{' >> gpurun_out/r3aa_ab.log
}
for rep in 1 2; do
  run tools/ab/liblcbase.so 4
  run tools/ab/liblc252.so 4
  run tools/ab/liblc128.so 4
  run tools/ab/liblc128.so 5
done
