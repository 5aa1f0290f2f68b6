# lanes sweep on the GPU box: GPU batch tests, then bench at 8 pairs/GPU
tools/gpu_step.sh 300 gpurun_out/ln_tests.log python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread && \
tools/gpu_step.sh 200 gpurun_out/ln_l1.log python bench.py --pairs 8 --lanes 1 --no-cpu-baseline --no-profile && \
tools/gpu_step.sh 200 gpurun_out/ln_l2.log python bench.py --pairs 8 --lanes 2 --no-cpu-baseline --no-profile && \
tools/gpu_step.sh 200 gpurun_out/ln_l3.log python bench.py --pairs 8 --lanes 3 --no-cpu-baseline --no-profile && \
tools/gpu_step.sh 200 gpurun_out/ln_l4.log python bench.py --pairs 8 --lanes 4 --no-cpu-baseline --no-profile && \
OF_BIG_PX=400000 tools/gpu_step.sh 200 gpurun_out/ln_l3b.log python bench.py --pairs 8 --lanes 3 --no-cpu-baseline --no-profile && \
OF_BIG_PX=3000000 tools/gpu_step.sh 200 gpurun_out/ln_l3c.log python bench.py --pairs 8 --lanes 3 --no-cpu-baseline --no-profile
