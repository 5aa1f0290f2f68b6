# GPU tests + bench at 1, 2, 3 lanes
tools/gpu_step.sh 400 gpurun_out/ck_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
tools/gpu_step.sh 300 gpurun_out/ck_bench1.log python bench.py --lanes 1 --no-cpu-baseline && \
tools/gpu_step.sh 300 gpurun_out/ck_bench2.log python bench.py --lanes 2 --no-cpu-baseline --no-profile && \
tools/gpu_step.sh 300 gpurun_out/ck_bench3.log python bench.py --lanes 3 --no-cpu-baseline --no-profile && \
tools/gpu_step.sh 300 gpurun_out/ck_bench3b.log python bench.py --lanes 3 --no-cpu-baseline --no-profile && \
tools/gpu_step.sh 300 gpurun_out/ck_bench4.log python bench.py --lanes 4 --no-cpu-baseline --no-profile
