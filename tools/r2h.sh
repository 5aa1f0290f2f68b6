set -u
timeout -k 10 60 tools/micro/wmf_phases > gpurun_out/r2h_phases.log 2>&1 && \
tools/gpu_step.sh 120 gpurun_out/r2h_wmf3.log python tools/wmf_bench.py --reps 10 && \
tools/gpu_step.sh 120 gpurun_out/r2h_wmf1.log python tools/wmf_bench.py --gc 1 --reps 10 && \
tools/gpu_step.sh 300 gpurun_out/r2h_tests.log python -u -m pytest tests/test_gpu_stages.py -v -s -x --timeout 120 --timeout-method thread -k "median"
