"""Middlebury flow colour coding (host-side; reference: optical_flow/viz/flow_color.py)."""
import numpy as np


def make_colorwheel():
    segs = [(15, (255, None, 0)), (6, (None, 255, 0)), (4, (0, 255, None)),
            (11, (0, None, 255)), (13, (None, 0, 255)), (6, (255, 0, None))]
    rows = []
    for s, (n, spec) in enumerate(segs):
        ramp = np.floor(255 * np.arange(n) / n)
        block = np.zeros((n, 3))
        for c in range(3):
            if spec[c] is None:
                block[:, c] = ramp if (s % 2 == 0) else 255 - ramp
            else:
                block[:, c] = spec[c]
        rows.append(block)
    return np.concatenate(rows, axis=0)


def compute_color(u, v):
    wheel = make_colorwheel()
    ncols = wheel.shape[0]
    rad = np.sqrt(u * u + v * v)
    a = np.arctan2(-v, -u) / np.pi
    fk = (a + 1) / 2.0 * (ncols - 1)
    k0 = np.floor(fk).astype(int)
    k1 = k0 + 1
    k1[k1 == ncols] = 0
    f = fk - k0
    img = np.zeros(u.shape + (3,), dtype=np.uint8)
    for i in range(3):
        col = wheel[k0, i] / 255.0 * (1 - f) + wheel[k1, i] / 255.0 * f
        col = 1 - rad * (1 - col)
        col[rad > 1] = col[rad > 1] * 0.75
        img[:, :, i] = np.floor(255 * np.clip(col, 0, 1)).astype(np.uint8)
    return img


def flow_to_color(flow, max_flow=None):
    """(H, W, 3) uint8 Middlebury colour image; |u| or |v| > 1e9 is unknown
    (black).  Arithmetic stays in the flow's own dtype (float32 flows are
    coloured in float32, as the reference does)."""
    u = np.array(flow[:, :, 0])
    v = np.array(flow[:, :, 1])
    unknown = (np.abs(u) > 1e9) | (np.abs(v) > 1e9)
    if max_flow is not None:
        max_rad = max_flow
    else:
        known = ~unknown
        max_rad = np.sqrt(u[known] ** 2 + v[known] ** 2).max() if np.any(known) else 0.0
    max_rad = max(max_rad, 1e-8)
    img = compute_color(u / max_rad, v / max_rad)
    img[unknown] = 0
    return img
