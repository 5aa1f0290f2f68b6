#!/bin/bash
set -u
export PYTHONDONTWRITEBYTECODE=1
bash tools/r4_final.sh r4y tests && bash tools/r4_prof.sh r4y && bash tools/r4_final.sh r4y bench
