# round-1 re-check of the tree with k_cgs: GPU tests, smoke, bench, rocprofv3 passes
mkdir -p gpurun_out
tools/gpu_step.sh 500 gpurun_out/r1e_tests.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread && \
tools/gpu_step.sh 200 gpurun_out/r1e_smoke.log python -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh 400 gpurun_out/r1e_bench.log python bench.py && \
bash tools/profile.sh r1e
