"""RubberWhale parity vs the 'backslash' surrogate tolerance (GPU)."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-python_amd"))
from PIL import Image
from optical_flow.methods.config import load_of_method
from optical_flow.io.flo_io import read_flo
from optical_flow.evaluation.metrics import flow_angular_error as fae
import optical_flow.interface as itf
G = os.path.join(ROOT, "tests", "golden")
im1 = np.array(Image.open(os.path.join(G, "frame10.png"))).astype(float)
im2 = np.array(Image.open(os.path.join(G, "frame11.png"))).astype(float)
gt = read_flo(os.path.join(G, "flow10.flo"))
ref = np.load(os.path.join(G, "rubberwhale_ref.npz"))
for method in ("classic+nl-fast", "hs-brightness"):
    r = ref[method].astype(float)
    a_ref = fae(gt[..., 0], gt[..., 1], r[..., 0], r[..., 1])
    for rtol in [float(x) for x in sys.argv[1:]]:
        t = time.time()
        uv = itf.estimate_flow(im1, im2, method, {"backslash_rtol": rtol})
        dt = time.time() - t
        a = fae(gt[..., 0], gt[..., 1], uv[..., 0], uv[..., 1])
        e = np.sqrt(((uv - r) ** 2).sum(-1))
        print(json.dumps({"method": method, "rtol": rtol, "sec": round(dt, 3), "dAEPE": a[2] - a_ref[2],
                          "dAAE": a[0] - a_ref[0], "aepe": a[2], "aepe_ref": a_ref[2], "mean": float(e.mean()),
                          "median": float(np.median(e)), "p99": float(np.percentile(e, 99)), "max": float(e.max())}),
              flush=True)
