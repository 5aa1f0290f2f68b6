"""Occlusion confidence on the GPU (reference: optical_flow/utils/occlusion.py:6-56)."""
import numpy as np

from optical_flow import _native as nat


def detect_occlusion(uv, images, sigma_d=0.3, sigma_i=20.0):
    """exp(-div^2/2sd^2) * exp(-|I2(x+u)-I1|^2/2si^2)."""
    if sigma_d != 0.3 or sigma_i != 20.0:
        raise NotImplementedError("detect_occlusion runs with the reference defaults sigma_d=0.3, sigma_i=20")
    uv = np.asarray(uv, dtype=float)
    images = np.asarray(images, dtype=float)
    H, W = uv.shape[:2]
    nc = images.shape[2] // 2
    out = np.empty((H, W), dtype=np.float32)
    ctx = nat.context()
    ctx.check(ctx.lib.of_detect_occlusion(ctx.handle, nat.ptr(nat.planar(uv)), nat.ptr(nat.planar(images)),
                                          H, W, nc, nat.ptr(out)))
    return out.astype(float)
