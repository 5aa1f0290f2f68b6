# lanes sweep of the host-to-host bench (no profiled replay, no CPU baseline), 2 reps
set -e
: > gpurun_out/lanes_ab.log
for rep in 1 2; do for L in 2 3 4; do
  echo "== lanes $L rep $rep" >> gpurun_out/lanes_ab.log
  timeout -k 10 200 python bench.py --lanes $L --no-cpu-baseline --no-profile 2>/dev/null | grep '^{' >> gpurun_out/lanes_ab.log
done; done
