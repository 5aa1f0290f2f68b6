"""What is the chaotic family's GPU-vs-reference gap made of? (VERDICT r4
item 2.)  The fp64 oracle (tests' checker) is run end to end on the
e2e_synth pair (synth_pair(120, 160, 0), tests/golden/e2e_synth.npz) with its
'backslash' PCG stopped at several relative residuals (oracle knob
ofr_set_backslash_rtol; 1e-12 = the oracle's spsolve restatement), and the
flow compared with the reference's own (golden) flow.  fp64 arithmetic
throughout, so any gap that grows with rtol is the surrogate's stopping
point, not fp32.  Then the same with every solution rounded to float32 (oracle
knob ofr_set_round_x_f32: what the GPU's fp32 x alone does).  The reference's
own spread under 1e-12 / 6e-8 input perturbations (chaos_synth.npz) is
printed beside.
usage: python tools/rtol_chaos.py [--f32-only] [methods...]  -> JSON lines"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'optical-flow-python_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')]
import oracle as O  # noqa: E402
from conftest import epe_stats  # noqa: E402

G = os.path.join(ROOT, 'tests', 'golden')


def main():
    args = sys.argv[1:]
    # --f32-only: only the runs with every solution rounded to float32
    f32_only = "--f32-only" in args
    methods = [a for a in args if not a.startswith("--")] or ['classic-c', 'classic++']
    rtols = [] if f32_only else [1e-12, 1e-9, 1e-8, 1e-7, 3e-7, 1e-6, 3e-6]
    rtols_f32 = [1e-12, 1e-8, 1e-6]
    d = np.load(os.path.join(G, 'e2e_synth.npz'))
    ch = np.load(os.path.join(G, 'chaos_synth.npz'))
    for m in methods:
        ref = d[m] if m in d else ch[m]
        spread = {eps: [float(ch[f"{m}:eps{eps}:seed{k}:mean"]) for k in range(3)] for eps in ("1e-12", "6e-08")}
        runs = [(r, False) for r in rtols] + [(r, True) for r in rtols_f32]
        for rtol, f32 in runs:
            O.set_backslash_rtol(rtol)
            O.set_round_x_f32(f32)
            uv = O.estimate_flow(d['im1'], d['im2'], m)
            s = epe_stats(uv, ref)
            print(json.dumps({"method": m, "oracle_rtol": rtol, "x_rounded_to_f32": f32, "mean": s["mean"],
                              "median": s["median"], "p99": s["p99"], "ref_spread_mean": spread}), flush=True)
        O.set_backslash_rtol(None)
        O.set_round_x_f32(False)


if __name__ == '__main__':
    main()
