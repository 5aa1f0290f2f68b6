#!/bin/bash
# round 3: token slots x k_cgs blocks x lanes sweep (host-to-host bench, 2 reps)
set -e
: > gpurun_out/r3z_ab.log
run() {  # lib lanes
  echo "== $1 lanes $2 rep $rep" >> gpurun_out/r3z_ab.log
  OPTFLOW_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --lanes $2 2>/dev/null | grep '^{' >> gpurun_out/r3z_ab.log
}
for rep in 1 2; do
  run tools/ab/libs2b252.so 3
  run tools/ab/libs2b252.so 4
  run tools/ab/libs2b252.so 5
  run tools/ab/libs2b200.so 4
  run tools/ab/libs3b168.so 4
  run tools/ab/libs3b168.so 5
  run tools/ab/libs4b128.so 5
  run tools/ab/libs4b128.so 6
done
