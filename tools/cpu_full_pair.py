"""Time the float64 C oracle (OpenMP, test infrastructure) on ONE full
1920x1080 Classic+NL-fast pair on the GPU box's host cores, to check the
bench's bounded-crop cpu_baseline extrapolation against a full-size run.
usage: python tools/cpu_full_pair.py > gpurun_out/cpu_full.json"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "optical-flow-python_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from optical_flow.utils.synthetic import synth_pair  # noqa: E402

im1, im2, gt = synth_pair(1080, 1920, 0)
t0 = time.perf_counter()
uv = oracle.estimate_flow(im1, im2, "classic+nl-fast")
dt = time.perf_counter() - t0
aepe = float((((uv - gt) ** 2).sum(-1) ** 0.5).mean())
print(json.dumps({"kind": "port", "what": "float64 C oracle estimate_flow('classic+nl-fast') on synth_pair(1080,1920,0)",
                  "seconds": round(dt, 2), "pairs_per_s": 1.0 / dt, "cores": oracle.num_threads(), "aepe_gt": aepe}))
