#!/bin/bash
set -u
export PYTHONDONTWRITEBYTECODE=1
bash tools/r4_prof.sh r4z && \
bash tools/r4_final.sh r4z bench
