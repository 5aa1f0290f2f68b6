# GPU tests + bench (serial lanes=1 and default lanes) with kernel profile
tools/gpu_step.sh 400 gpurun_out/ck_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
tools/gpu_step.sh 300 gpurun_out/ck_bench1.log python bench.py --lanes 1 --no-cpu-baseline && \
tools/gpu_step.sh 300 gpurun_out/ck_bench.log python bench.py --no-cpu-baseline --no-profile
