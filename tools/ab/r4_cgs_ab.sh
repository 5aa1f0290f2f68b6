#!/bin/bash
# round 4: k_cgs with register rings for the records of waves 2 and 3 only
# (lib_cgs_rr23.so, 188 VGPRs) vs LDS record reads: isolated per-launch time at
# 1080p, bitwise flow check, and the headline bench
set -u
OUT=gpurun_out/r4_cgs_ab.log
: > $OUT
for rep in 1 2; do
for L in optical-flow-python_amd/optical_flow/_lib/liboptflow.so tools/ab/lib_cgs_rr23.so; do
  echo "== $L rep $rep" >> $OUT
  OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/pcg_bench.py --iters 200 2>&1 | grep '"variant"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']['pcg_iter']; print('k_cgs 1080p us/launch', round(k['ms_per_launch']*1e3,2), 'rel_res', d['rel_res'])" >> $OUT || exit 1
  if [ $rep = 1 ]; then
    OPTFLOW_LIB=$L timeout -k 10 120 python -u tools/ab/bitwise.py 540 960 >> $OUT 2>&1 || exit 1
  fi
  OPTFLOW_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-profile --no-cpu-baseline > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json >> $OUT; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('headline pairs/s', d['value'], 'host', d['host_to_host']['value'])" >> $OUT
done
done
