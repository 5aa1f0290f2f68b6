"""estimate_flow (reference: optical_flow/interface.py:11-141).

RGB -> gray (uint8 round trip) and RGB -> Lab (+ per-channel [0,255]
scaling) run on the GPU inside of_estimate_flow, followed by the whole
coarse-to-fine schedule; one C call per pair."""
import ctypes as C

import numpy as np

from optical_flow import _abi
from optical_flow import _native as nat
from optical_flow.methods.config import load_of_method


def estimate_flow(im1, im2, method='classic+nl-fast', params=None):
    """Flow (H, W, 2) float64 from im1 to im2; (H, W) or (H, W, >=3) inputs."""
    im1 = np.asarray(im1, dtype=float)
    im2 = np.asarray(im2, dtype=float)
    ope = load_of_method(method)
    if params is not None:
        ope.parse_input_parameter(params)
    H, W = im1.shape[:2]
    if im1.ndim == 3 and im1.shape[2] < 3:
        # interface.py:47: channels are concatenated, no colour conversion
        ope.images = np.concatenate([im1, im2], axis=2)
        if ope.color_images is not None:
            ope.color_images = im1.copy()
        return ope.compute_flow(np.zeros((H, W, 2)))
    if im1.ndim == 3:
        a = nat.f32(im1[:, :, :3])
        b = nat.f32(im2[:, :, :3])
        Cc = 3
    else:
        a, b, Cc = nat.f32(im1), nat.f32(im2), 1
    P = ope.to_params()
    P.guide_mode = int(ope._METHOD == 'classic_nl' and ope.color_images is not None)
    out = np.empty((2, H, W), dtype=np.float32)
    st = _abi.OfStats()
    ctx = nat.context()
    ctx.check(ctx.lib.of_estimate_flow(ctx.handle, C.byref(P), nat.ptr(a), nat.ptr(b), H, W, Cc, None,
                                       nat.ptr(out), C.byref(st)))
    ope.alpha = P.alpha
    ope.last_stats = st.as_dict()
    return nat.interleaved(out)


def _preprocess(im1, im2):
    a = nat.f32(np.asarray(im1, dtype=float)[:, :, :3])
    b = nat.f32(np.asarray(im2, dtype=float)[:, :, :3])
    H, W = a.shape[:2]
    gray = np.empty((2, H, W), dtype=np.float32)
    lab = np.empty((3, H, W), dtype=np.float32)
    ctx = nat.context()
    ctx.check(ctx.lib.of_preprocess(ctx.handle, nat.ptr(a), nat.ptr(b), H, W, nat.ptr(gray), nat.ptr(lab)))
    return gray, lab


def _rgb2gray(im):
    """MATLAB double(rgb2gray(uint8(im))) on the GPU (interface.py:74-88)."""
    im = np.asarray(im, dtype=float)
    if im.ndim == 2:
        return im
    return _preprocess(im, im)[0][0].astype(float)


def _rgb2lab_scaled(im):
    """_rgb2lab (interface.py:91-141) followed by the per-channel scale_image
    to [0, 255] that estimate_flow applies (interface.py:58-61)."""
    return nat.interleaved(_preprocess(im, im)[1])
