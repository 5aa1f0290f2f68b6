# A/B of k_cgs builds: fixed-iteration CG timing at 1080p and 540p, twice
# (rel_res must agree bitwise between builds of the same arithmetic)
# usage: bash tools/ab/ab.sh LIB...
set -e
mkdir -p gpurun_out
: > gpurun_out/ab_pcg.log
for i in 1 2; do
for L in "$@"; do
  echo "== $L" >> gpurun_out/ab_pcg.log
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/pcg_bench.py --iters 200 >> gpurun_out/ab_pcg.log 2>&1
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/pcg_bench.py --h 540 --w 960 --iters 200 >> gpurun_out/ab_pcg.log 2>&1
done; done
