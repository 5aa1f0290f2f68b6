#!/bin/bash
# round-3 check + WMF fp32 chunk-sum A/B
set -u
export PYTHONDONTWRITEBYTECODE=1
tools/gpu_step.sh 600 gpurun_out/r3m_gpu.log python -u -m pytest -v -rA --timeout 300 --timeout-method thread tests -m gpu && \
tools/gpu_step.sh 200 gpurun_out/r3m_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh 300 gpurun_out/r3m_wmf32_tests.log env OPTFLOW_LIB=tools/ab/libwmf32.so python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_stages.py tests/test_gpu_e2e.py -m gpu -k "weighted_median or wmf or e2e" && \
bash tools/ab/bench_ab.sh tools/ab/libwmf64.so tools/ab/libwmf32.so && \
tools/gpu_step.sh 400 gpurun_out/r3m_bench.log python -u bench.py
