#!/bin/bash
# round 4: pipelined-SOR variants (publication interval G, waves per CU) on
# config 2 (hs + sor, 480x640, 8 pairs, 4 lanes): pairs/s and the flow's sha1
set -u
OUT=gpurun_out/r4_sor_ab.log
: > $OUT
for L in optical-flow-python_amd/optical_flow/_lib/liboptflow.so tools/ab/lib_sor_G4S32.so tools/ab/lib_sor_G8S16.so; do
  echo "== $L" >> $OUT
  OPTFLOW_LIB=$L timeout -k 10 200 python -u bench.py --method hs --solver sor --height 480 --width 640 --steps 2 \
      --warmup 1 --no-profile --no-cpu-baseline > /tmp/b.json 2>&1 || { echo "bench failed $?" >> $OUT; tail -3 /tmp/b.json >> $OUT; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('pairs/s', d['value'], 'levels', [l['ms'] for l in d['ms_per_level']])" >> $OUT
  OPTFLOW_LIB=$L timeout -k 10 120 python -u - >> $OUT 2>&1 <<'PY' || exit 1
import hashlib, os, sys
sys.path.insert(0, "optical-flow-python_amd")
import numpy as np, optical_flow
from optical_flow.utils.synthetic import synth_pair
im1, im2, _ = synth_pair(480, 640, 0)
uv = optical_flow.estimate_flow(im1.astype(np.uint8), im2.astype(np.uint8), "hs", {"solver": "sor"})
print("sha1", hashlib.sha1(np.ascontiguousarray(uv).tobytes()).hexdigest())
PY
done
