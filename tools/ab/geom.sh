# CG convergence at geometries with tall bands (R = 64): default build and the
# CGS_TARGET_BLOCKS=320 build that diverged at 1080p
set -e
L=optical-flow-python_amd/optical_flow/_lib/liboptflow.so
: > gpurun_out/geom.log
for hw in "1792 1920" "1080 3360" "1080 1920"; do set -- $hw
  echo "== main $1 $2" >> gpurun_out/geom.log
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/pcg_bench.py --h $1 --w $2 --iters 200 >> gpurun_out/geom.log 2>&1
done
for hw in "1080 1920" "1088 1920" "1024 1920"; do set -- $hw
  echo "== tb320old $1 $2" >> gpurun_out/geom.log
  OPTFLOW_LIB=tools/ab/tb320old.so timeout -k 10 120 python -u tools/pcg_bench.py --h $1 --w $2 --iters 200 >> gpurun_out/geom.log 2>&1
  echo "== tb320 $1 $2" >> gpurun_out/geom.log
  OPTFLOW_LIB=tools/ab/tb320.so timeout -k 10 120 python -u tools/pcg_bench.py --h $1 --w $2 --iters 200 >> gpurun_out/geom.log 2>&1
done
