"""Weighted median filtering (reference: optical_flow/utils/weighted_median.py)."""
import numpy as np

from optical_flow import _native as nat


def weighted_median_1d(w, u):
    """Smallest sorted u whose cumulative weight reaches half the total
    (weighted_median.py:5-21).  Host utility; the filter below runs on GPU."""
    idx = np.argsort(u)
    cw = np.cumsum(np.asarray(w, dtype=float)[idx])
    k = np.searchsorted(cw, cw[-1] / 2.0)
    return np.asarray(u)[idx][min(k, len(u) - 1)]


def median_filter2(a, size):
    """scipy.ndimage.median_filter(a, size, mode='reflect') on the GPU, for a
    2-D array or an (H, W, C) stack filtered per channel."""
    a = np.asarray(a, dtype=float)
    p = nat.planar(a)
    out = np.empty_like(p)
    ctx = nat.context()
    ctx.check(ctx.lib.of_median_filter(ctx.handle, nat.ptr(p), a.shape[0], a.shape[1], p.shape[0], int(size),
                                       nat.ptr(out)))
    return out[0].astype(float) if a.ndim == 2 else nat.interleaved(out)


def denoise_color_weighted_medfilt2(uv, color_images, occ, area_hsz, mfsz, sigma_i, full_version=False):
    """Colour-guided, occlusion-weighted median over a (2*area_hsz+1)^2 window
    (weighted_median.py:24-112); plain median when there is no guide."""
    uv = np.asarray(uv, dtype=float)
    H, W = uv.shape[:2]
    if color_images is None or np.asarray(color_images).size < H * W:
        sz = int(mfsz[0]) if hasattr(mfsz, '__len__') else int(mfsz)
        return median_filter2(uv, sz)
    g = np.asarray(color_images, dtype=float)
    if g.shape[0] != H or g.shape[1] != W:
        raise NotImplementedError("colour guide of a different size (skimage resize path)")
    gp = nat.planar(g)
    out = np.empty((2, H, W), dtype=np.float32)
    ctx = nat.context()
    ctx.check(ctx.lib.of_weighted_median(ctx.handle, nat.ptr(nat.planar(uv)), nat.ptr(gp), gp.shape[0],
                                         nat.ptr(nat.f32(occ)), H, W, int(area_hsz), float(sigma_i), nat.ptr(out)))
    return nat.interleaved(out)
