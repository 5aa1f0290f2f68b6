tools/gpu_step.sh 900 gpurun_out/gpu_tests.log python -m pytest tests -m gpu -x -q && \
tools/gpu_step.sh 300 gpurun_out/rw.log python -m pytest tests/test_gpu_e2e.py -k rubberwhale -s -q && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1h.log 2>&1
