# coarse-level CG: k_cgs launches vs the one-workgroup k_cg_small solve at
# 68x120 and 135x240 (30 iterations, fixed count)
set -e
: > gpurun_out/small.log
for L in optical-flow-python_amd/optical_flow/_lib/liboptflow.so tools/ab/sm8192.so tools/ab/sm32768.so; do
for hw in "68 120" "135 240"; do set -- $hw
  echo "== $L $1 $2" >> gpurun_out/small.log
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/pcg_bench.py --h $1 --w $2 --iters 30 >> gpurun_out/small.log 2>&1
done; done
