# full GPU check of the tree: -m gpu tests, smoke, default bench (TAG names the logs)
set -u
TAG=${1:-run}
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
tools/gpu_step.sh 900 gpurun_out/${TAG}_gpu.log python -u -m pytest -v -rA --timeout 300 --timeout-method thread tests -m gpu && \
tools/gpu_step.sh 200 gpurun_out/${TAG}_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh 400 gpurun_out/${TAG}_bench.log python -u bench.py
