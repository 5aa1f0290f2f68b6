#!/bin/bash
# round-4 SOR check: pipelined-vs-per-sweep bitwise tests, reference SOR
# tests, the config-2 full-size test, the hook GPU test, config-2 bench
set -u
TAG=${1:-r4a}
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
tools/gpu_step.sh 400 gpurun_out/${TAG}_sor_tests.log python -u -m pytest -v -rA --timeout 200 --timeout-method thread \
    tests/test_gpu_stages.py -k "sor" && \
tools/gpu_step.sh 300 gpurun_out/${TAG}_hook.log python -u -m pytest -v -rA --timeout 200 --timeout-method thread \
    tests/test_reference_hook.py -m gpu && \
tools/gpu_step.sh 400 gpurun_out/${TAG}_cfg2_test.log python -u -m pytest -v -rA --timeout 300 --timeout-method thread \
    tests/test_gpu_fullsize.py -k "cfg2" && \
tools/gpu_step.sh 300 gpurun_out/${TAG}_bench_cfg2.log python -u bench.py --method hs --solver sor --height 480 --width 640
