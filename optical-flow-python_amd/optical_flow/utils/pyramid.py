"""Gaussian pyramids on the GPU (reference: optical_flow/utils/pyramid.py:6-73)."""
import ctypes as C

import numpy as np

from optical_flow import _native as nat


def _matlab_round(x):
    return int(np.floor(x + 0.5))


def compute_image_pyramid(img, f, n_levels, ratio):
    """Level k+1 = imresize(correlate(level k, f, 'reflect'), ratio), bilinear,
    MATLAB coordinates (pyramid.py:44-73).  Index 0 = finest."""
    img = np.asarray(img, dtype=float)
    f = np.asarray(f, dtype=float)
    if f.ndim != 2 or f.shape[0] != f.shape[1] or f.shape[0] % 2 == 0:
        raise NotImplementedError("pyramid smoothing kernel must be odd and square")
    pyr = [img.copy()]
    cur = nat.planar(img)
    H, W = img.shape[:2]
    ctx = nat.context()
    kern = np.ascontiguousarray(f, dtype=np.float64)
    for _ in range(1, n_levels):
        nH, nW = max(1, _matlab_round(H * ratio)), max(1, _matlab_round(W * ratio))
        out = np.empty((cur.shape[0], nH, nW), dtype=np.float32)
        oh, ow = C.c_int(0), C.c_int(0)
        ctx.check(ctx.lib.of_pyramid_level(ctx.handle, nat.ptr(cur), H, W, cur.shape[0], nat.dptr(kern),
                                           f.shape[0], float(ratio), nat.ptr(out), C.byref(oh), C.byref(ow)))
        cur, H, W = out, nH, nW
        pyr.append(out[0].astype(float) if img.ndim == 2 else nat.interleaved(out))
    return pyr
