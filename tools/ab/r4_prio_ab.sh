#!/bin/bash
# round 4: k_cgs waves 1 / 3 at issue priority 1 (lib_cgs_prio.so) vs 0
# (in-tree): the timed rate (HBM-resident value and host to host), 3 reps
set -u
OUT=gpurun_out/r4_prio_ab.log
: > $OUT
for rep in 1 2 3; do
for L in optical-flow-python_amd/optical_flow/_lib/liboptflow.so tools/ab/lib_cgs_prio.so; do
  echo "== $L rep $rep" >> $OUT
  OPTFLOW_LIB=$L timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-profile --no-cpu-baseline --no-stream > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json >> $OUT; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('pairs/s', d['value'], 'host', d['host_to_host']['value'])" >> $OUT
done
done
