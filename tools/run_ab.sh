# A/B of the CG kernels on the GPU box (tests, fixed-iteration kernel timing, bench)
tools/gpu_step.sh 400 gpurun_out/ab_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
tools/gpu_step.sh 120 gpurun_out/ab_pcg3.log python tools/pcg_bench.py && \
OF_CG_WAVES=768 tools/gpu_step.sh 120 gpurun_out/ab_pcg3w768.log python tools/pcg_bench.py && \
OF_CG_POLY=1 tools/gpu_step.sh 120 gpurun_out/ab_pcg1.log python tools/pcg_bench.py && \
OF_CG_POLY=1 OF_CG_WAVES=1024 tools/gpu_step.sh 120 gpurun_out/ab_pcg1w1024.log python tools/pcg_bench.py && \
tools/gpu_step.sh 200 gpurun_out/ab_bench3.log python bench.py --no-cpu-baseline
