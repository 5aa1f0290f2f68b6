timeout -k 10 120 python tools/pcg_bench.py > gpurun_out/pcgab.log 2>&1 || exit $?
timeout -k 10 120 python tools/pcg_bench.py --solver pcg >> gpurun_out/pcgab.log 2>&1 || exit $?
tools/gpu_step.sh 900 gpurun_out/gpu_tests.log python -m pytest tests -m gpu -x -q && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1g.log 2>&1
