# lexicographic SOR A/B: per-sweep time at 480x640 / 240x320 per library build
set -e
: > gpurun_out/sor_ab.log
for L in "$@"; do for hw in "480 640" "240 320"; do
  set -- $hw
  echo "== $L $1x$2" >> gpurun_out/sor_ab.log
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/pcg_bench.py --solver sor --h $1 --w $2 --iters 200 2>&1 | grep '"variant"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernels']['sor_sweep']['ms_per_launch']*1e3,1), 'us/sweep', d['iters'], d['rel_res'])" >> gpurun_out/sor_ab.log
done; done
