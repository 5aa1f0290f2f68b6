# lanes A/B round 3: token at 2-3 lanes vs serial, 3 reps
for rep in 1 2 3; do
  OF_BIG_PX=1048576 tools/gpu_step.sh 200 gpurun_out/ln_t2.$rep.log python bench.py --pairs 8 --lanes 2 --no-cpu-baseline --no-profile || exit $?
  OF_BIG_PX=1048576 tools/gpu_step.sh 200 gpurun_out/ln_t3.$rep.log python bench.py --pairs 8 --lanes 3 --no-cpu-baseline --no-profile || exit $?
  tools/gpu_step.sh 200 gpurun_out/ln_s1.$rep.log python bench.py --pairs 8 --lanes 1 --no-cpu-baseline --no-profile || exit $?
done
