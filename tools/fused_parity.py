"""Fused warp + assembly vs the two-kernel form, against the references:
mean / median EPE to the fp64 oracle (smoke pair) and to the reference's
golden flows (e2e_small crop, e2e_synth), per method, each form.
usage (GPU box): python tools/fused_parity.py  -> JSON lines"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'optical-flow-python_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')]
import optical_flow  # noqa: E402
import oracle as O  # noqa: E402
from conftest import epe_stats  # noqa: E402
from optical_flow import _abi, _native  # noqa: E402
from optical_flow.utils.synthetic import synth_pair  # noqa: E402

G = os.path.join(ROOT, 'tests', 'golden')


def main():
    ctx = _native.context()
    cases = []
    im1, im2, _ = synth_pair(48, 64, seed=3)
    cases.append(("smoke48x64", im1, im2, {"classic+nl-fast": O.estimate_flow(im1, im2, "classic+nl-fast")}))
    d = np.load(os.path.join(G, 'e2e_small.npz'))
    cases.append(("e2e_small", d['im1'], d['im2'], {m: d[m] for m in ("classic+nl-fast", "hs", "ba", "classic-c")}))
    s = np.load(os.path.join(G, 'e2e_synth.npz'))
    cases.append(("e2e_synth", s['im1'], s['im2'], {m: s[m] for m in ("classic+nl-fast", "hs", "classic-c")}))
    for name, a, b, refs in cases:
        for m, ref in refs.items():
            out = {"case": name, "method": m}
            for fused in (1, 0):
                ctx.set_option(_abi.OF_OPT_FUSED_WARP, fused)
                st = epe_stats(optical_flow.estimate_flow(a, b, m), ref)
                out["fused" if fused else "two_kernels"] = {k: round(v, 7) for k, v in st.items()}
            ctx.set_option(_abi.OF_OPT_FUSED_WARP, 1)
            print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
