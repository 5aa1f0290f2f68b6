#!/bin/bash
# round 6: config 3 (Classic-C + 'pcg', 720p) rocprofv3 trace + PMC passes at
# the shipped k_cg geometry (640 waves per launch), summarised on the box into
# profiles/pmc_traffic.json, then the config-3 bench line that reads it
set -u
export PYTHONDONTWRITEBYTECODE=1
tools/profile.sh r6c3 --method classic-c --solver pcg --height 720 --width 1280 || exit $?
python tools/prof_summary.py gpurun_out/prof_r6c3 --H 720 --W 1280 --traffic --workload classic-c@720x1280/pcg \
  --source r6c3 > gpurun_out/prof_r6c3/summary.txt 2>&1 || exit $?
cp profiles/pmc_traffic.json gpurun_out/prof_r6c3/pmc_traffic.json
# only summaries travel back (gpurun merges <= 64 MiB of gpurun_out/)
rm -f gpurun_out/prof_r6c3/*_kernel_trace.csv gpurun_out/prof_r6c3/*_counter_collection.csv
tools/gpu_step.sh 300 gpurun_out/prof_r6c3/bench_cfg3.log python -u bench.py --method classic-c --solver pcg --height 720 --width 1280
