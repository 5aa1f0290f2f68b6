#!/bin/bash
set -u
export PYTHONDONTWRITEBYTECODE=1
tools/gpu_step.sh 300 gpurun_out/r4n_4k.log python -u -m pytest -v -rA -s --timeout 250 --timeout-method thread tests/test_gpu_fullsize.py -k 4k -m gpu && \
bash tools/r4_final.sh r4n tests
