#!/bin/bash
# round-4 validation: every -m gpu test, smoke, the default bench and the
# configs 2 / 3 bench lines, the file pipeline bench (TAG names the logs)
set -u
TAG=${1:-r4f}
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
tools/gpu_step.sh 1100 gpurun_out/${TAG}_gpu.log python -u -m pytest -v -rA --timeout 300 --timeout-method thread tests -m gpu && \
tools/gpu_step.sh 200 gpurun_out/${TAG}_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh 400 gpurun_out/${TAG}_bench.log python -u bench.py && \
tools/gpu_step.sh 300 gpurun_out/${TAG}_bench_cfg2.log python -u bench.py --method hs --solver sor --height 480 --width 640 && \
tools/gpu_step.sh 300 gpurun_out/${TAG}_bench_cfg3.log python -u bench.py --method classic-c --solver pcg --height 720 --width 1280 && \
tools/gpu_step.sh 400 gpurun_out/${TAG}_pipeline.log python -u tools/pipeline_bench.py --pairs 48
