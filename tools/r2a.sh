set -u
export PYTHONDONTWRITEBYTECODE=1
tools/gpu_step.sh 300 gpurun_out/r2a_sor.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stages.py -k "sor or library" && \
tools/gpu_step.sh 900 gpurun_out/r2a_gpu.log python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu && \
tools/gpu_step.sh 400 gpurun_out/r2a_bench.log python -u bench.py --no-cpu-baseline
