#!/bin/bash
set -u
export PYTHONDONTWRITEBYTECODE=1
bash tools/r4_final.sh r4s tests && tools/gpu_step.sh 400 gpurun_out/r4s_bench.log python -u bench.py
