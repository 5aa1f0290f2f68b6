#!/bin/bash
# pipeline stream reuse + HBM-resident bench value
set -u
export PYTHONDONTWRITEBYTECODE=1
tools/gpu_step.sh 300 gpurun_out/r4g_tests.log python -u -m pytest -v -rA --timeout 200 --timeout-method thread tests/test_pipeline.py tests/test_gpu_batch.py -m gpu && \
tools/gpu_step.sh 400 gpurun_out/r4g_bench.log python -u bench.py && \
tools/gpu_step.sh 300 gpurun_out/r4g_pipeline.log python -u tools/pipeline_bench.py --pairs 48
