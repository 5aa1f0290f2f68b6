tools/gpu_step.sh 900 gpurun_out/gpu_tests.log python -m pytest tests -m gpu -x -q && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1f.log 2>&1
