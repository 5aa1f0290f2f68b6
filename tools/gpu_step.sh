#!/bin/bash
# run one GPU step under its own time limit; print its exit code; return
# non-zero only for crash-like exits (fault/abort/segv/timeout) so callers
# can chain steps with && and stop after anything worse than a test failure.
# usage: tools/gpu_step.sh SECONDS LOGFILE cmd...
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "EXIT $rc" >> "$log"
case $rc in
  0|1|5) exit 0 ;;   # success / test failures / no tests collected
  *) echo "step failed hard (rc=$rc): $*"; exit $rc ;;
esac
