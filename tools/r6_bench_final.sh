#!/bin/bash
# round 6: the shipped tree's bench lines -- default `python bench.py` (K 10,
# W 2) twice, the driver's form (--steps 20 --warmup 5), --rccl-self
set -u
TAG=${1:-r6bench}
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
tools/gpu_step.sh 300 $O/bench_default1.log python -u bench.py && \
tools/gpu_step.sh 300 $O/bench_default2.log python -u bench.py && \
tools/gpu_step.sh 300 $O/bench_k20.log python -u bench.py --gpus 1 --steps 20 --warmup 5 && \
tools/gpu_step.sh 300 $O/bench_rccl_self.log python -u bench.py --rccl-self
