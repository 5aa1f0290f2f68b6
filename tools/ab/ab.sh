set -e
mkdir -p gpurun_out
: > gpurun_out/ab_pcg.log
for i in 1 2; do
for L in tools/ab/remap.so optical-flow-python_amd/optical_flow/_lib/liboptflow.so; do
  echo "== $L" >> gpurun_out/ab_pcg.log
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/pcg_bench.py --iters 200 >> gpurun_out/ab_pcg.log 2>&1
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/pcg_bench.py --h 540 --w 960 --iters 200 >> gpurun_out/ab_pcg.log 2>&1
done; done
