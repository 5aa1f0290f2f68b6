#!/bin/bash
set -u
export PYTHONDONTWRITEBYTECODE=1
OPTFLOW_LIB=tools/ab/lib_wmf_halves.so tools/gpu_step.sh 300 gpurun_out/r4t_halves_tests.log python -u -m pytest -v -rA --timeout 200 --timeout-method thread tests/test_gpu_stages.py tests/test_gpu_e2e.py -k "weighted_median or median_filter or small_crop or rubberwhale or synthetic" -m gpu && tools/ab/r4_wmf_ab.sh
