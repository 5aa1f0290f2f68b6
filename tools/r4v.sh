#!/bin/bash
# run-to-run spread of the default bench line on one box (5 runs)
set -u
export PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/r4v_spread.log
: > $OUT
for rep in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --no-profile --no-cpu-baseline > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json >> $OUT; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('pairs/s', d['value'], 'host', d['host_to_host']['value'], 'streamed', d['streamed']['value'])" >> $OUT
done
