#!/bin/bash
set -u
export PYTHONDONTWRITEBYTECODE=1
tools/ab/r4_wmf_ab.sh && tools/ab/r4_cgs_ab.sh
