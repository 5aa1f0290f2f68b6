#!/bin/bash
# round 4: HIP hardware queues per process (GPU_MAX_HW_QUEUES, box default 4)
# x lanes: the timed rate, 2 reps
set -u
OUT=gpurun_out/r4_queues_ab.log
: > $OUT
for rep in 1 2; do
for cfg in "4 4" "8 4" "8 5" "8 8"; do
  set -- $cfg
  echo "== queues $1 lanes $2 rep $rep" >> $OUT
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --lanes $2 --no-profile --no-cpu-baseline --no-stream > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json >> $OUT; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('pairs/s', d['value'], 'host', d['host_to_host']['value'])" >> $OUT
done
done
