# weighted median A/B: k_wmf (old) vs k_wmf2 at 1080p, bitwise comparison, GPU stage tests
tools/gpu_step.sh 120 gpurun_out/wmf_old.log env OF_WMF_VARIANT=old python tools/wmf_bench.py --save gpurun_out/wmf_old.npy && \
tools/gpu_step.sh 120 gpurun_out/wmf_new.log python tools/wmf_bench.py --save gpurun_out/wmf_new.npy && \
tools/gpu_step.sh 120 gpurun_out/wmf_old1.log env OF_WMF_VARIANT=old python tools/wmf_bench.py --gc 1 --save gpurun_out/wmf_old1.npy && \
tools/gpu_step.sh 120 gpurun_out/wmf_new1.log python tools/wmf_bench.py --gc 1 --save gpurun_out/wmf_new1.npy && \
tools/gpu_step.sh 300 gpurun_out/wmf_tests.log python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_e2e.py -x -q --timeout 120 --timeout-method thread
