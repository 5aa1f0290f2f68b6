#!/bin/bash
# round 4: issue priority of the other lanes' kernels beside the fine CG:
# in-tree (all 0), lib_prio1 (warp / assembly / update at 1), lib_prio2
# (weighted median at 1); timed rate, 3 reps
set -u
OUT=gpurun_out/r4_prio2_ab.log
: > $OUT
for rep in 1 2 3; do
for L in optical-flow-python_amd/optical_flow/_lib/liboptflow.so tools/ab/lib_prio1.so tools/ab/lib_prio2.so; do
  echo "== $L rep $rep" >> $OUT
  OPTFLOW_LIB=$L timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-profile --no-cpu-baseline --no-stream > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json >> $OUT; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('pairs/s', d['value'], 'host', d['host_to_host']['value'])" >> $OUT
done
done
