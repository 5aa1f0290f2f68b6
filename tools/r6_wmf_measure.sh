#!/bin/bash
# round 6: the shipped weighted median measured -- per-phase clock64 stamps
# (tools/micro/wmf_phases, built with WMF_PHASE_TIMING from the same source)
# and the SQ instruction counters of one serial 1080p pair
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r6wmf; mkdir -p $O
tools/gpu_step.sh 120 $O/phases.log tools/micro/wmf_phases && \
tools/pmc_wmf_sq.sh r6wmf
