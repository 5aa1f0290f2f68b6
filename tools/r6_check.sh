#!/bin/bash
# round-6 validation in one gpurun call: every -m gpu test + smoke, then the
# default bench and its --rccl-self proxy (the N > 1 timed path at one rank)
set -u
TAG=${1:-r6}
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
tools/gpu_step.sh 700 gpurun_out/${TAG}_gpu.log python -u -m pytest -v -rA --timeout 300 --timeout-method thread tests -m gpu && \
tools/gpu_step.sh 150 gpurun_out/${TAG}_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh 200 gpurun_out/${TAG}_bench.log python -u bench.py --steps 20 --warmup 2 && \
tools/gpu_step.sh 200 gpurun_out/${TAG}_bench_rself.log python -u bench.py --steps 20 --warmup 2 --rccl-self
