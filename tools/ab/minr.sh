# coarse-level k_cgs band height A/B: fixed-iteration CG timing at the coarse
# 1080p pyramid sizes, then the host-to-host bench, per library build
set -e
: > gpurun_out/minr_ab.log
for L in "$@"; do
  for hw in "270 480" "135 240" "68 120" "540 960"; do
    set -- $hw
    echo "== $L $1x$2" >> gpurun_out/minr_ab.log
    OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/pcg_bench.py --h $1 --w $2 --iters 50 2>&1 | grep '"variant"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernels']['pcg_iter']['ms_per_launch']*1e3,2), 'us/launch', d['iters'])" >> gpurun_out/minr_ab.log
  done
done
