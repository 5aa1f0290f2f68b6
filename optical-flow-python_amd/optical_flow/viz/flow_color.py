"""Middlebury flow colour coding on the GPU (reference:
optical_flow/viz/flow_color.py:5-107).

flow_to_color runs as two HIP kernels behind of_flow_to_color
(include/optflow.h): the largest known radius, then the per-pixel wheel map.
The arithmetic keeps numpy's dtype rules (float32 flows are normalised and
placed on the wheel in float32, as the reference does; float64 otherwise), so
the image equals the reference's (tests/test_gpu_viz.py).  No CPU fallback.
"""
import ctypes as C

import numpy as np

from optical_flow import _native as nat


def flow_to_color(flow, max_flow=None):
    """(H, W, 3) uint8 Middlebury colour image of an (H, W, 2) flow; |u| or
    |v| > 1e9 is unknown (black); normalised by max(max_flow, 1e-8), or by
    the largest known radius when max_flow is None."""
    flow = np.asarray(flow)
    if flow.ndim != 3 or flow.shape[2] < 2:
        raise ValueError("flow must be (H, W, 2)")
    dt = np.float32 if flow.dtype == np.float32 else np.float64
    f = np.ascontiguousarray(flow[:, :, :2], dtype=dt)
    H, W = f.shape[:2]
    out = np.zeros((H, W, 3), dtype=np.uint8)
    ctx = nat.context()
    ctx.check(ctx.lib.of_flow_to_color(ctx.handle, f.ctypes.data_as(C.c_void_p), 0 if dt == np.float32 else 1,
                                       H, W, int(max_flow is not None),
                                       float(max_flow) if max_flow is not None else 0.0,
                                       out.ctypes.data_as(C.c_void_p)))
    return out
