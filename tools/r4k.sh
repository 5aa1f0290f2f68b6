#!/bin/bash
set -u
export PYTHONDONTWRITEBYTECODE=1
tools/ab/r4_prio_ab.sh && \
tools/gpu_step.sh 300 gpurun_out/r4k_pipeline.log python -u tools/pipeline_bench.py --pairs 48
