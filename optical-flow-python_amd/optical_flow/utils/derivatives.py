"""Spatio-temporal derivatives with warping on the GPU
(reference: optical_flow/utils/derivatives.py:148-296)."""
import numpy as np

from optical_flow import _abi
from optical_flow import _native as nat


def partial_deriv(images, uv, interp_method='cubic', deriv_filter=None, blend=0.5):
    """It, Ix, Iy of frame 2 warped by uv against frame 1.  'bi-cubic' =
    Hermite bicubic with analytic derivatives, 'cubic' = cubic B-spline,
    'bi-linear' = bilinear."""
    if deriv_filter is None:
        deriv_filter = np.array([1, -8, 0, 8, -1]) / 12.0
    if interp_method not in _abi.INTERP:
        raise ValueError(f"Unknown interpolation method: {interp_method}")
    filt = np.ascontiguousarray(np.asarray(deriv_filter, dtype=float).ravel())
    if filt.size != 5:
        raise NotImplementedError("deriv_filter must have 5 taps")
    images = np.asarray(images, dtype=float)
    H, W, Cc = images.shape
    nc = Cc // 2
    outs = [np.empty((nc, H, W), dtype=np.float32) for _ in range(3)]
    ctx = nat.context()
    ctx.check(ctx.lib.of_partial_deriv(ctx.handle, nat.ptr(nat.planar(images)), H, W, nc,
                                       nat.ptr(nat.planar(uv)), _abi.INTERP[interp_method], nat.dptr(filt),
                                       float(blend), *[nat.ptr(o) for o in outs]))
    if Cc == 2:
        return tuple(o[0].astype(float) for o in outs)
    return tuple(nat.interleaved(o) for o in outs)
