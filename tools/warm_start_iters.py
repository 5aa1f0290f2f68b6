"""Warm-starting the 'backslash' solve, measured in the fp64 oracle before
building it (VERDICT r5 "next" 2).

The reference's default solver is SuperLU (`spsolve`, base.py:107-108): its
answer does not depend on a starting iterate, so the GPU's CG surrogate may
start anywhere and must only reach the same 1e-6 relative residual.  Here the
oracle's 'backslash' PCG (2x2 block Jacobi, stopped at ||r|| < 1e-6 ||b||,
the GPU surrogate's criterion) runs Classic+NL-fast on synth_pair(H, W, 0)
with each starting iterate of ofr_set_warm_start for the warps after a
level's first (a level's first warp starts from 0 in every mode):
  0   x0 = 0 (as shipped)
  1   the previous warp's unclipped solution
  2   (uv_prev + x_prev) - uv: what the weighted median took back of the
      previous step
  11, 12  the same directions scaled by the A-norm optimal gamma
Prints one JSON line per mode: iterations per solve, the robust stage's fine
solves, totals, and the flow's AEPE / distance to mode 0's flow.

    python tools/warm_start_iters.py [--height 540 --width 960] [--modes 0,1,2,11,12]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "optical-flow-python_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402  (test infrastructure: the fp64 restatement)
from optical_flow.utils.synthetic import synth_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=540)
    ap.add_argument("--width", type=int, default=960)
    ap.add_argument("--modes", default="0,1,2,11,12")
    ap.add_argument("--rtol", type=float, default=1e-6)
    a = ap.parse_args()
    im1, im2, gt = synth_pair(a.height, a.width, 0)
    oracle.set_backslash_rtol(a.rtol)
    base = None
    for mode in [int(m) for m in a.modes.split(",")]:
        oracle.set_warm_start(mode)
        oracle.solve_log()
        t0 = time.perf_counter()
        uv = oracle.estimate_flow(im1, im2, "classic+nl-fast")
        dt = time.perf_counter() - t0
        log = oracle.solve_log()
        if base is None:
            base = uv
        fine = max(h * w for h, w, *_ in log)
        robust = [it for h, w, i, it, al in log if al < 0.5]
        rec = {"size": [a.height, a.width], "mode": mode, "rtol": a.rtol, "seconds": round(dt, 1),
               "iters_total": sum(r[3] for r in log),
               "iters_robust_stage": sum(robust),
               "iters_fine_levels": sum(r[3] for r in log if r[0] * r[1] >= fine * 0.5),
               "iters_warp1": sum(r[3] for r in log if r[2] == 0),
               "iters_warp2_3": sum(r[3] for r in log if r[2] > 0),
               "per_solve": [[h, w, i, it, al] for h, w, i, it, al in log],
               "aepe_gt": round(float(np.sqrt(((uv - gt) ** 2).sum(-1)).mean()), 6),
               "epe_to_mode0_mean": float(np.sqrt(((uv - base) ** 2).sum(-1)).mean())}
        print(json.dumps(rec), flush=True)
    oracle.set_warm_start(0)
    oracle.set_backslash_rtol(None)


if __name__ == "__main__":
    main()
