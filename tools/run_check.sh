# GPU tests + bench (1 and 2 lanes; profile on the serial one)
tools/gpu_step.sh 400 gpurun_out/ck_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
tools/gpu_step.sh 300 gpurun_out/ck_bench1.log python bench.py --lanes 1 --no-cpu-baseline && \
tools/gpu_step.sh 300 gpurun_out/ck_bench2.log python bench.py --no-cpu-baseline --no-profile && \
tools/gpu_step.sh 300 gpurun_out/ck_bench2b.log python bench.py --no-cpu-baseline --no-profile
