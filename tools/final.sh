#!/bin/bash
# validation of a tree in two calls (each under gpurun's 1200 s):
#   tools/final.sh TAG tests  -> every -m gpu test + smoke
#   tools/final.sh TAG bench  -> default bench, configs 2 / 3, file pipeline
set -u
TAG=${1:-final}
PART=${2:-tests}
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
if [ "$PART" = tests ]; then
tools/gpu_step.sh 1000 gpurun_out/${TAG}_gpu.log python -u -m pytest -v -rA --timeout 300 --timeout-method thread tests -m gpu && \
tools/gpu_step.sh 150 gpurun_out/${TAG}_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
else
tools/gpu_step.sh 400 gpurun_out/${TAG}_bench.log python -u bench.py && \
tools/gpu_step.sh 250 gpurun_out/${TAG}_bench_cfg2.log python -u bench.py --method hs --solver sor --height 480 --width 640 && \
tools/gpu_step.sh 250 gpurun_out/${TAG}_bench_cfg3.log python -u bench.py --method classic-c --solver pcg --height 720 --width 1280 && \
tools/gpu_step.sh 300 gpurun_out/${TAG}_pipeline.log python -u tools/pipeline_bench.py --pairs 48
fi
