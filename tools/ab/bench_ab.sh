# host-to-host bench A/B of two library builds (no profiled replay, no CPU baseline), 2 reps each
set -e
: > gpurun_out/bench_ab.log
for rep in 1 2; do for L in "$@"; do
  echo "== $L rep $rep" >> gpurun_out/bench_ab.log
  OPTFLOW_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile 2>/dev/null | grep '^{' >> gpurun_out/bench_ab.log
done; done
