"""Flow resampling on the GPU (reference: optical_flow/utils/warping.py:6-45)."""
import numpy as np

from optical_flow import _native as nat


def resample_flow(uv, target_sz, method='bilinear'):
    """Bilinear resize; BOTH components scale by the height ratio (warping.py:25-26)."""
    uv = np.asarray(uv, dtype=float)
    H, W = uv.shape[:2]
    nH, nW = int(target_sz[0]), int(target_sz[1])
    if (H, W) == (nH, nW):
        return uv.copy()
    out = np.empty((2, nH, nW), dtype=np.float32)
    ctx = nat.context()
    ctx.check(ctx.lib.of_resample_flow(ctx.handle, nat.ptr(nat.planar(uv)), H, W, nH, nW, nat.ptr(out)))
    return nat.interleaved(out)
