# FETCH_SIZE / WRITE_SIZE of k_cgs on the fixed-iteration 1080p CG bench (one pass each)
# usage: bash tools/ab/pmc_cgs.sh LIB TAG
set -e
export TMPDIR=/tmp
L=$1; T=$2; OUT=gpurun_out/pmc_cgs_$T
mkdir -p $OUT
OPTFLOW_LIB=$L tools/gpu_step.sh 120 $OUT/fetch.log rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_cgs -f csv -d $OUT -o fetch -- python3 tools/pcg_bench.py --iters 50
OPTFLOW_LIB=$L tools/gpu_step.sh 120 $OUT/write.log rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_cgs -f csv -d $OUT -o write -- python3 tools/pcg_bench.py --iters 50
