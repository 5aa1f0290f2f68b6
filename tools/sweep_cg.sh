#!/bin/bash
# A/B sweep of the CG knobs (Chebyshev interval lower end, k_cgs block count)
# and lane count on the default 1080p bench; one bench process per setting,
# each under its own time limit; stops at the first failure.
set -e
mkdir -p gpurun_out/sweep
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-profile --steps 6 --warmup 1 $BENCH_ARGS \
    > gpurun_out/sweep/$tag.log 2>&1
  echo "$tag $(grep '^{' gpurun_out/sweep/$tag.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("solver_iters_total"), d.get("aepe_gt"))')"
}
for a in ${CHEB_SWEEP:-0.04 0.06 0.08 0.10 0.12 0.15}; do run cheb$a OF_CG_CHEB_A=$a; done
