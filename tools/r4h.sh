#!/bin/bash
set -u
export PYTHONDONTWRITEBYTECODE=1
tools/gpu_step.sh 400 gpurun_out/r4h_bench.log python -u bench.py && \
tools/gpu_step.sh 300 gpurun_out/r4h_pipeline.log python -u tools/pipeline_bench.py --pairs 48 && \
tools/gpu_step.sh 200 gpurun_out/r4h_pipe_tests.log python -u -m pytest -v -rA --timeout 150 --timeout-method thread tests/test_pipeline.py -m gpu && \
tools/ab/r4_wmf_ab.sh
