#!/bin/bash
# GPU check: -m gpu tests, smoke, bench (TAG names the logs; extra args go to bench.py)
set -u
TAG=$1; shift
export PYTHONDONTWRITEBYTECODE=1
tools/gpu_step.sh 600 gpurun_out/${TAG}_gpu.log python -u -m pytest -v -rA --timeout 300 --timeout-method thread tests -m gpu && \
tools/gpu_step.sh 200 gpurun_out/${TAG}_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh 400 gpurun_out/${TAG}_bench.log python -u bench.py "$@"
