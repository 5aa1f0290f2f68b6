# Chebyshev interval sweep: bench (1 pair, serial) per lower bound a
for a in 0.04 0.01 0.02 0.03 0.06 0.08; do
  OF_CG_CHEB_A=$a tools/gpu_step.sh 200 gpurun_out/cheb_$a.log python bench.py --pairs 2 --lanes 1 --steps 2 --no-cpu-baseline --no-profile || exit $?
done
