#!/bin/bash
# HBM traffic and duration A/B of library builds for some kernels (one serial
# 1080p pair: kernel trace, FETCH_SIZE pass, WRITE_SIZE pass per library),
# then the default bench per library (2 reps).  Summarise each directory
# with tools/prof_summary.py gpurun_out/TAG/<i>.
# usage: tools/ab/traffic_ab.sh TAG 'KERNEL_REGEX' LIB...
set -u
TAG=$1; KRE=$2; shift 2
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
S="bench.py --steps 1 --warmup 0 --pairs 1 --lanes 1 --no-cpu-baseline --no-profile --no-stream"
i=0
for L in "$@"; do
  D=$O/$i; mkdir -p $D; echo "$L" > $D/lib.txt
  OPTFLOW_LIB=$L tools/gpu_step.sh 300 $D/trace1.log rocprofv3 --kernel-trace --stats -f csv -d $D -o trace1 -- python3 $S || exit $?
  OPTFLOW_LIB=$L tools/gpu_step.sh 300 $D/fetch.log rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $D -o fetch -- python3 $S || exit $?
  OPTFLOW_LIB=$L tools/gpu_step.sh 300 $D/write.log rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $D -o write -- python3 $S || exit $?
  gzip -f $D/*_trace.csv
  i=$((i+1))
done
for rep in 1 2; do for L in "$@"; do
  echo "== $L rep $rep" >> $O/bench_ab.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 300 $O/bench_tmp.log python -u bench.py --steps 6 --no-cpu-baseline --no-profile || exit $?
  grep '^{' $O/bench_tmp.log >> $O/bench_ab.log
done; done
