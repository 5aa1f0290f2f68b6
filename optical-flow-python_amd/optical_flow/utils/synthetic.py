"""Deterministic synthetic image pairs with analytic ground-truth flow.

numpy-only so the GPU box can regenerate the benchmark inputs without scipy.
Recipe follows SURVEY.md §8(d) (``synth_pair``): per RGB channel, K=32 plane
waves; frame 2 samples the same field at (x - u, y - v); ground truth
u = 2 sin(2*pi*y/H) + 0.5, v = 1.5 cos(2*pi*x/W) - 0.25.
"""
import numpy as np


def _field(x, y, f, th, ph):
    K = f.shape[1]
    out = np.empty(x.shape + (3,))
    for c in range(3):
        acc = np.zeros(x.shape)
        for k in range(K):
            acc += np.sin(f[c, k] * (x * np.cos(th[c, k]) + y * np.sin(th[c, k])) + ph[c, k])
        out[..., c] = 128.0 + 40.0 * acc / np.sqrt(K)
    return out


def synth_gt(H, W):
    """Analytic ground-truth flow (H, W, 2) for :func:`synth_pair`."""
    y, x = np.mgrid[0:H, 0:W].astype(float)
    u = 2.0 * np.sin(2.0 * np.pi * y / H) + 0.5
    v = 1.5 * np.cos(2.0 * np.pi * x / W) - 0.25
    return np.stack([u, v], axis=2)


def synth_pair(H, W, seed=0, K=32):
    """Return (im1, im2, gt) — two float64 RGB frames with integer values in
    [0, 255] and the (H, W, 2) ground-truth flow from frame 1 to frame 2."""
    rng = np.random.default_rng(seed)
    f = rng.uniform(0.03, 0.35, size=(3, K))
    th = rng.uniform(0.0, 2.0 * np.pi, size=(3, K))
    ph = rng.uniform(0.0, 2.0 * np.pi, size=(3, K))
    y, x = np.mgrid[0:H, 0:W].astype(float)
    gt = synth_gt(H, W)
    i1 = _field(x, y, f, th, ph)
    i2 = _field(x - gt[..., 0], y - gt[..., 1], f, th, ph)
    im1 = np.floor(np.clip(i1, 0, 255) + 0.5)
    im2 = np.floor(np.clip(i2, 0, 255) + 0.5)
    return im1, im2, gt
