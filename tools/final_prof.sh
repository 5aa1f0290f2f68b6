#!/bin/bash
# profiles of the default bench (final tree of a round): rocprofv3 kernel traces (timed lanes
# and isolated), PMC passes, then the summaries committed under profiles/
set -u
TAG=${1:-final}
export PYTHONDONTWRITEBYTECODE=1
tools/profile.sh $TAG || exit $?
D=gpurun_out/prof_$TAG
python3 tools/prof_summary.py $D --traffic --workload "classic+nl-fast@1080x1920/backslash" --source "$TAG" > $D/summary.txt 2>&1 && \
python3 tools/inner_loop_rocprof.py $D/trace1_kernel_trace.csv > $D/inner_loop.json 2>&1 && \
python3 tools/side_by_side_rocprof.py $D/trace_kernel_trace.csv $D/side_by_side.json > $D/side_by_side.txt 2>&1 && \
cp profiles/pmc_traffic.json $D/pmc_traffic.json
