"""Image processing utilities (reference: optical_flow/utils/image_processing.py).

scale_image / fspecial_gaussian are tiny host helpers (kernel weights and a
linear map); structure_texture_decomposition_rof runs on the GPU."""
import ctypes as C

import numpy as np

from optical_flow import _native as nat


def scale_image(im, vlow, vhigh, ilow=None, ihigh=None):
    """Linear rescale to [vlow, vhigh] (image_processing.py:6-26)."""
    im = np.asarray(im, dtype=float)
    lo = im.min() if ilow is None else ilow
    hi = im.max() if ihigh is None else ihigh
    if hi == lo:
        return np.full_like(im, (vlow + vhigh) / 2.0)
    return (im - lo) / (hi - lo) * (vhigh - vlow) + vlow


def fspecial_gaussian(size, sigma):
    """MATLAB fspecial('gaussian') (image_processing.py:29-49)."""
    if isinstance(size, (int, np.integer)):
        size = (int(size), int(size))
    m, n = [(s - 1) / 2.0 for s in size]
    y, x = np.ogrid[-m:m + 1, -n:n + 1]
    h = np.exp(-(x * x + y * y) / (2.0 * sigma * sigma))
    h[h < np.finfo(h.dtype).eps * h.max()] = 0
    s = h.sum()
    return h / s if s != 0 else h


def structure_texture_decomposition_rof(im, theta=1.0 / 8, n_iters=100, alp=0.95):
    """ROF structure-texture split on the GPU (image_processing.py:52-136)."""
    im = np.asarray(im, dtype=float)
    H, W = im.shape[:2]
    p = nat.planar(im)
    out = np.empty_like(p)
    ctx = nat.context()
    ctx.check(ctx.lib.of_rof_texture(ctx.handle, nat.ptr(p), H, W, p.shape[0], float(theta), int(n_iters),
                                     float(alp), nat.ptr(out)))
    return out[0].astype(float) if im.ndim == 2 else nat.interleaved(out)
