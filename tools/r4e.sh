set -u
export PYTHONDONTWRITEBYTECODE=1
T="python -u -m pytest -v -rA --timeout 300 --timeout-method thread"
tools/gpu_step.sh 400 gpurun_out/r4e_tests.log $T tests/test_gpu_stages.py tests/test_gpu_reference_cases.py tests/test_gpu_e2e.py tests/test_reference_hook.py tests/test_gpu_filters.py -m gpu -k "not rubberwhale" && \
tools/ab/r4_cgs_ab.sh && \
tools/gpu_step.sh 300 gpurun_out/r4e_altba_probe.log python -u tools/altba_gpu_probe.py && \
tools/ab/r4_sor_ab.sh
