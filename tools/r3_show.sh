#!/bin/bash
# summarise a tools/r3_check2.sh run
TAG=$1
grep -E "passed|failed" gpurun_out/${TAG}_gpu.log | tail -1; grep FAILED gpurun_out/${TAG}_gpu.log; tail -2 gpurun_out/${TAG}_smoke.log
grep "^{" gpurun_out/${TAG}_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('pairs/s', d['value'], 'host', d['host_to_host']['value'], 'roof', r['frac'], 'finest', r['finest']['frac'], 'inner', r['inner_loop']['frac'], 'iters', d['solver_iters_total'])
print(d['kernel_ms_per_pair_isolated']); print(d['ms_per_level'])"
