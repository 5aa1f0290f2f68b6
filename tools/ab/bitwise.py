"""sha1 of the Classic+NL-fast flow of synth_pair(H, W, 0) with the library
OPTFLOW_LIB names (A/B builds that must agree bitwise)."""
import hashlib, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "optical-flow-python_amd"))
import numpy as np
import optical_flow
from optical_flow.utils.synthetic import synth_pair
H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1080, 1920)
im1, im2, _ = synth_pair(H, W, 0)
uv = optical_flow.estimate_flow(im1.astype(np.uint8), im2.astype(np.uint8), "classic+nl-fast")
print(os.environ.get("OPTFLOW_LIB", "default"), H, W, hashlib.sha1(np.ascontiguousarray(uv).tobytes()).hexdigest())
