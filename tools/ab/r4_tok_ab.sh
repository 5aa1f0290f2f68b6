#!/bin/bash
# round 4: fine-solve token slots x blocks per side-by-side solve at 4 lanes:
# in-tree 2 x 252, lib_tok3x168 (3 x 168), lib_tok3x200 (3 x 200); timed rate
set -u
OUT=gpurun_out/r4_tok_ab.log
: > $OUT
for rep in 1 2; do
for L in optical-flow-python_amd/optical_flow/_lib/liboptflow.so tools/ab/lib_tok3x168.so tools/ab/lib_tok3x200.so; do
  echo "== $L rep $rep" >> $OUT
  OPTFLOW_LIB=$L timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-profile --no-cpu-baseline --no-stream > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json >> $OUT; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('pairs/s', d['value'], 'host', d['host_to_host']['value'], 'same flow', d['host_to_host']['host_flow_equals_timed_flow'])" >> $OUT
done
done
