#!/bin/bash
# pool on the context's own lanes: batch / pipeline GPU tests, the ordering
# probe, two default bench lines
set -u
TAG=${1:-r5j}
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
tools/gpu_step.sh 400 $O/tests.log python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_batch.py tests/test_pipeline.py -m gpu || exit $?
tools/gpu_step.sh 300 $O/probe.log python -u tools/order_probe.py 8 || exit $?
for rep in 1 2; do
  tools/gpu_step.sh 300 $O/bench$rep.log python -u bench.py --steps 20 --no-cpu-baseline --no-profile || exit $?
done
