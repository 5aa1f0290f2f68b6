# SQ stall breakdown of the CG kernels (tools/pcg_bench.py, 1080p, 200 iterations)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_cg
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS"
tools/gpu_step.sh 120 gpurun_out/pmc_cg/p3.log rocprofv3 --pmc $C --kernel-include-regex "k_cg" -f csv -d gpurun_out/pmc_cg -o p3 -- python3 tools/pcg_bench.py --iters 50 && \
OF_CG_POLY=1 tools/gpu_step.sh 120 gpurun_out/pmc_cg/p1.log rocprofv3 --pmc $C --kernel-include-regex "k_cg" -f csv -d gpurun_out/pmc_cg -o p1 -- python3 tools/pcg_bench.py --iters 50 && \
tools/gpu_step.sh 120 gpurun_out/pmc_cg/t3.log python3 tools/pcg_bench.py
