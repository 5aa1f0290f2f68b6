#!/bin/bash
set -u
export PYTHONDONTWRITEBYTECODE=1
OPTFLOW_LIB=tools/ab/lib_wmf_shift.so tools/gpu_step.sh 200 gpurun_out/r4j_wmf_tests.log python -u -m pytest -v -rA --timeout 150 --timeout-method thread tests/test_gpu_stages.py -k "weighted_median or median_filter" -m gpu && \
tools/ab/r4_wmf_ab.sh && \
bash tools/r4_final.sh r4j bench
