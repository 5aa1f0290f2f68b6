#!/bin/bash
# round 3 final: rocprofv3 passes of the default bench (tools/profile.sh),
# the occupancy timeline of the trace, configs 2 / 3 bench lines
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
TAG=$1
bash tools/profile.sh $TAG || exit $?
f=$(find gpurun_out/prof_$TAG -name "trace_kernel_trace.csv" | head -1)
python3 tools/timeline.py $f --win-ms 100 > gpurun_out/prof_$TAG/timeline.txt || true
tools/gpu_step.sh 300 gpurun_out/${TAG}_bench_cfg2.log python -u bench.py --method hs --solver sor --height 480 --width 640 && \
tools/gpu_step.sh 300 gpurun_out/${TAG}_bench_cfg3.log python -u bench.py --method classic-c --solver pcg --height 720 --width 1280
