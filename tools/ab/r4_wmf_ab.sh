#!/bin/bash
# round 4: WMF two waves per tile with the window rows split (k_wmf3,
# lib_wmf_halves.so) vs k_wmf (in-tree): isolated 1080p WMF launch time (bench lanes=1 replay),
# the headline, and the flow's sha1 (k_wmf3 rounds the chunk sums differently)
set -u
OUT=gpurun_out/r4_wmf_ab.log
: > $OUT
for rep in 1 2; do
for L in optical-flow-python_amd/optical_flow/_lib/liboptflow.so tools/ab/lib_wmf_halves.so; do
  echo "== $L rep $rep" >> $OUT
  if [ $rep = 1 ]; then
    OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/ab/bitwise.py 540 960 >> $OUT 2>&1 || exit 1
  fi
  OPTFLOW_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json >> $OUT; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('pairs/s', d['value'], 'host', d['host_to_host']['value'], 'wmf ms/launch', r['wmf']['mean_launch_ms'], 'wmf ms/pair', d['kernel_ms_per_pair_isolated'].get('wmf'), 'cg us', round(r['finest']['mean_launch_ms']*1e3,2))" >> $OUT
done
done
