#!/bin/bash
# round-5 check: re-run the tests changed after r5g, queue-mapping probes,
# then bench A/B of three builds (previous commit / specialised assembly,
# two kernels / fused warp + assembly), 2 reps each
set -u
TAG=${1:-r5h}
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
tools/gpu_step.sh 300 $O/tests.log python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_display.py tests/test_gpu_stages.py -m gpu -k "fused or display or stage_report or prints" || exit $?
tools/gpu_step.sh 300 $O/probe_dedicated.log python -u tools/order_probe.py 8 || exit $?
OF_STREAM_QUEUE=shared tools/gpu_step.sh 300 $O/probe_shared.log python -u tools/order_probe.py 8 || exit $?
for rep in 1 2; do for L in build/ab/base.so build/ab/unfused.so build/ab/fused.so; do
  echo "== $L rep $rep" >> $O/bench_ab.log
  OPTFLOW_LIB=$L tools/gpu_step.sh 300 $O/bench_tmp.log python -u bench.py --steps 10 --no-cpu-baseline --no-profile || exit $?
  grep '^{' $O/bench_tmp.log >> $O/bench_ab.log
done; done
