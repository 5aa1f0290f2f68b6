"""Parity margin vs the 'backslash' surrogate tolerance (GPU): the smoke pair
(synth_pair(48,64,3)) and the e2e crop against the float64 oracle / the
reference, RubberWhale against the reference, and the CG iterations of one
1080p pair, per rtol.  usage: python tools/rtol_check.py 1e-6 5e-7 ..."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "optical-flow-python_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402  (checker only)
import optical_flow.interface as itf  # noqa: E402
from optical_flow.utils.synthetic import synth_pair  # noqa: E402
from PIL import Image  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
im1, im2, _ = synth_pair(48, 64, seed=3)
smoke_ref = oracle.estimate_flow(im1, im2, "classic+nl-fast")
e2e = np.load(os.path.join(G, "e2e_small.npz"))
rw1 = np.array(Image.open(os.path.join(G, "frame10.png"))).astype(float)
rw2 = np.array(Image.open(os.path.join(G, "frame11.png"))).astype(float)
rwref = np.load(os.path.join(G, "rubberwhale_ref.npz"))["classic+nl-fast"].astype(float)
b1, b2, _ = synth_pair(1080, 1920, 0)


def epe(a, b):
    return float(np.sqrt(((a - b) ** 2).sum(-1)).mean())


for rtol in [float(x) for x in sys.argv[1:]]:
    p = {"backslash_rtol": rtol}
    r = {"rtol": rtol,
         "smoke_mean": epe(itf.estimate_flow(im1, im2, "classic+nl-fast", p), smoke_ref),
         "crop_mean": epe(itf.estimate_flow(e2e["im1"], e2e["im2"], "classic+nl-fast", p), e2e["classic+nl-fast"]),
         "rubberwhale_mean": epe(itf.estimate_flow(rw1, rw2, "classic+nl-fast", p), rwref)}
    from optical_flow.methods.config import load_of_method  # noqa: E402
    t = time.time()
    o = load_of_method("classic+nl-fast")
    o.backslash_rtol = rtol
    uv = itf.estimate_flow(b1, b2, "classic+nl-fast", p)
    r["sec_1080p"] = round(time.time() - t, 3)
    print(json.dumps(r), flush=True)
