# k_cgs vs k_cgp: fixed-iteration kernel timing (+ residual), GPU tests, bench
tools/gpu_step.sh 120 gpurun_out/cgs_pcg.log python tools/pcg_bench.py && \
OF_CG_KERNEL=cgp tools/gpu_step.sh 120 gpurun_out/cgp_pcg.log python tools/pcg_bench.py && \
tools/gpu_step.sh 400 gpurun_out/cgs_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
tools/gpu_step.sh 300 gpurun_out/cgs_bench1.log python bench.py --lanes 1 --no-cpu-baseline && \
tools/gpu_step.sh 300 gpurun_out/cgs_bench2.log python bench.py --no-cpu-baseline --no-profile
