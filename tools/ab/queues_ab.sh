#!/bin/bash
# stream -> hardware-queue mapping A/B (dedicated CU-masked queues vs the
# runtime's shared pool) + the new-entry GPU tests + one default bench line
set -u
TAG=$1
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
tools/gpu_step.sh 400 $O/tests.log python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_display.py tests/test_gpu_batch.py tests/test_pipeline.py -m gpu || exit $?
tools/gpu_step.sh 400 $O/probe_dedicated.log python -u tools/order_probe.py 10 || exit $?
OF_STREAM_QUEUE=shared tools/gpu_step.sh 400 $O/probe_shared.log python -u tools/order_probe.py 10 || exit $?
tools/gpu_step.sh 300 $O/bench.log python -u bench.py --steps 20 --no-cpu-baseline --no-profile || exit $?
