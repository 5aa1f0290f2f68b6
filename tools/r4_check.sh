#!/bin/bash
# round-4 GPU check of the new pieces: pipelined SOR (bitwise vs per-sweep,
# reference SOR, config-2 full size), the reference hook, the general-filter
# solve log, the streaming pair pool, k_cg_reg without scratch (smoke), then
# the config-2 bench line
set -u
TAG=${1:-r4b}
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
T="python -u -m pytest -v -rA --timeout 300 --timeout-method thread"
tools/gpu_step.sh 400 gpurun_out/${TAG}_sor_tests.log $T tests/test_gpu_stages.py -k "sor" && \
tools/gpu_step.sh 300 gpurun_out/${TAG}_new_tests.log $T tests/test_reference_hook.py tests/test_pipeline.py \
    tests/test_gpu_filters.py tests/test_gpu_e2e.py -m gpu -k "not rubberwhale" && \
tools/gpu_step.sh 200 gpurun_out/${TAG}_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh 400 gpurun_out/${TAG}_cfg2_test.log $T tests/test_gpu_fullsize.py -k "cfg2" && \
tools/gpu_step.sh 300 gpurun_out/${TAG}_bench_cfg2.log python -u bench.py --method hs --solver sor --height 480 --width 640 && \
tools/gpu_step.sh 200 gpurun_out/${TAG}_altba_probe.log python -u tools/altba_gpu_probe.py
