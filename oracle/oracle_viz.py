"""Test infrastructure only: a numpy restatement of the reference's
flow_to_color (optical_flow/viz/flow_color.py:5-107), the checker of the HIP
path (of_flow_to_color, optical_flow.viz.flow_color).  Nothing in the
optical_flow package imports this file.

Pinned by tests/golden/viz_metrics.npz (images the reference itself made,
tests/golden/gen_golden.py gen_viz_metrics): bit-exact on every case
(tests/test_api_cpu.py).
"""
import numpy as np


def make_colorwheel():
    """flow_color.py:5-40: 55 bins, RY 15, YG 6, GC 4, CB 11, BM 13, MR 6;
    per segment one channel held at 255, one ramped up or down by
    floor(255 * k / n)."""
    segs = [(15, 0, 1, False), (6, 1, 0, True), (4, 1, 2, False),
            (11, 2, 1, True), (13, 2, 0, False), (6, 0, 2, True)]
    rows = []
    for n, hold, ramp, down in segs:
        r = np.floor(255 * np.arange(n) / n)
        block = np.zeros((n, 3))
        block[:, hold] = 255
        block[:, ramp] = 255 - r if down else r
        rows.append(block)
    return np.concatenate(rows, axis=0)


def compute_color(u, v, atan2_f32="numpy"):
    """flow_color.py:43-74 with numpy's dtype rules.  atan2_f32="rounded"
    takes float32 arctan2 as the float64 one rounded to float32 (what the
    device computes; numpy's own float32 arctan2 is a CPU-dependent vector
    routine that is not correctly rounded)."""
    wheel = make_colorwheel()
    ncols = wheel.shape[0]
    rad = np.sqrt(u ** 2 + v ** 2)
    if atan2_f32 == "rounded" and u.dtype == np.float32:
        at = np.arctan2((-v).astype(np.float64), (-u).astype(np.float64)).astype(np.float32)
    else:
        at = np.arctan2(-v, -u)
    a = at / np.pi
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


def flow_to_color(flow, max_flow=None, atan2_f32="numpy"):
    """flow_color.py:77-107: |u| or |v| > 1e9 is unknown (black); normalised
    by max(max_flow or the largest known radius, 1e-8)."""
    u = np.array(flow[:, :, 0])
    v = np.array(flow[:, :, 1])
    unknown = (np.abs(u) > 1e9) | (np.abs(v) > 1e9)
    if max_flow is not None:
        max_rad = max_flow
    else:
        known = ~unknown
        max_rad = np.sqrt(u[known] ** 2 + v[known] ** 2).max() if np.any(known) else 0.0
    max_rad = max(max_rad, 1e-8)
    img = compute_color(u / max_rad, v / max_rad, atan2_f32)
    img[unknown] = 0
    return img
