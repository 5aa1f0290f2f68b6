# weighted median timing at 1080p (+ output saved for comparison) and GPU stage/e2e tests
tools/gpu_step.sh 120 gpurun_out/wmf_new.log python tools/wmf_bench.py --save gpurun_out/wmf_new.npy && \
tools/gpu_step.sh 120 gpurun_out/wmf_new1.log python tools/wmf_bench.py --gc 1 --save gpurun_out/wmf_new1.npy && \
tools/gpu_step.sh 300 gpurun_out/wmf_tests.log python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_e2e.py -x -q --timeout 120 --timeout-method thread
