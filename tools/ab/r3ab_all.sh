#!/bin/bash
# round 3 check (tests, smoke, bench) then the coarse-block A/B
set -u
bash tools/r3_check2.sh r3z && bash tools/ab/r3aa.sh
