#!/bin/bash
# round-6 final validation of the tree: every -m gpu test + smoke, the
# default bench as the driver runs it, configs 2 and 3, the file pipeline
set -u
TAG=${1:-r6final}
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
tools/gpu_step.sh 700 $O/gpu_tests.log python -u -m pytest -v -rA --timeout 300 --timeout-method thread tests -m gpu && \
tools/gpu_step.sh 150 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh 300 $O/bench.log python -u bench.py && \
tools/gpu_step.sh 300 $O/bench_rccl_self.log python -u bench.py --rccl-self && \
tools/gpu_step.sh 250 $O/bench_cfg2.log python -u bench.py --method hs --solver sor --height 480 --width 640 && \
tools/gpu_step.sh 250 $O/bench_cfg3.log python -u bench.py --method classic-c --solver pcg --height 720 --width 1280 && \
tools/gpu_step.sh 300 $O/pipeline.log python -u tools/pipeline_bench.py --pairs 48
