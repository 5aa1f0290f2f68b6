# SQ instruction / stall breakdown of the weighted median kernel (tools/wmf_bench.py, 1080p)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_wmf
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS"
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA"

tools/gpu_step.sh 120 gpurun_out/pmc_wmf/p1.log timeout -s KILL 60 rocprofv3 --pmc $C1 --kernel-include-regex "k_wmf" -f csv -d gpurun_out/pmc_wmf -o p1 -- python3 tools/wmf_bench.py --reps 2 && \
tools/gpu_step.sh 120 gpurun_out/pmc_wmf/p2.log timeout -s KILL 60 rocprofv3 --pmc $C2 --kernel-include-regex "k_wmf" -f csv -d gpurun_out/pmc_wmf -o p2 -- python3 tools/wmf_bench.py --reps 2
