"""GPU side of tools/rtol_chaos.py: the chaotic family on the e2e_synth pair
(tests/golden/e2e_synth.npz) with the 'backslash' surrogate stopped at
several relative residuals (params {'backslash_rtol': ...}), distance to the
reference's own flow.  Compare with the fp64 oracle at the same rtol
(profiles/r5_rtol_chaos.jsonl): if the two agree, the gap to the reference
is the surrogate's stopping point, not fp32.
usage (GPU box): python tools/rtol_chaos_gpu.py  -> JSON lines"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'optical-flow-python_amd'), os.path.join(ROOT, 'tests')]
import optical_flow  # noqa: E402
from conftest import epe_stats  # noqa: E402

G = os.path.join(ROOT, 'tests', 'golden')


def main():
    d = np.load(os.path.join(G, 'e2e_synth.npz'))
    ch = np.load(os.path.join(G, 'chaos_synth.npz'))
    for m in ('classic-c', 'classic++'):
        ref = d[m] if m in d else ch[m]
        for rtol in (1e-6, 3e-7, 1e-7, 3e-8, 1e-8):
            uv = optical_flow.estimate_flow(d['im1'], d['im2'], m, {'backslash_rtol': rtol})
            s = epe_stats(uv, ref)
            print(json.dumps({"method": m, "gpu_rtol": rtol, "mean": s["mean"], "median": s["median"],
                              "p99": s["p99"], "finite": bool(np.isfinite(uv).all())}), flush=True)


if __name__ == '__main__':
    main()
