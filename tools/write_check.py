"""k_partial_deriv and k_flow_operator in isolation at 1080p (stage C
entries, 3 calls each) for a rocprofv3 --pmc WRITE_SIZE pass: compares their
write bytes outside the pipeline with the in-pipeline PMC numbers.
usage: rocprofv3 --pmc WRITE_SIZE ... -- python tools/write_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-python_amd"))
import numpy as np  # noqa: E402
from optical_flow.utils.derivatives import partial_deriv  # noqa: E402
from optical_flow.methods.config import load_of_method  # noqa: E402

H, W = 1080, 1920
rng = np.random.default_rng(0)
images = rng.uniform(0, 255, (H, W, 2))
uv = rng.normal(0, 1, (H, W, 2))
o = load_of_method("classic+nl-fast")
o.images = images
for _ in range(3):
    It, Ix, Iy = partial_deriv(images, uv, "bi-cubic")
for _ in range(3):
    o._operator_planes(uv, None, It, Ix, Iy, 0.0)
print("done")
