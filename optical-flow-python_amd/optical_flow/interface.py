"""estimate_flow (reference: optical_flow/interface.py:11-141).

RGB -> gray (uint8 round trip) and RGB -> Lab (+ per-channel [0,255]
scaling) run on the GPU inside of_estimate_flow, followed by the whole
coarse-to-fine schedule; one C call per pair."""
import ctypes as C

import numpy as np

from optical_flow import _abi
from optical_flow import _native as nat
from optical_flow.methods.base import progress_printer
from optical_flow.methods.config import load_of_method


def estimate_flow(im1, im2, method='classic+nl-fast', params=None, gt=None):
    """Flow (H, W, 2) float64 from im1 to im2; (H, W) or (H, W, >=3) inputs.
    Prints what the reference's compute_flow prints.  `gt` (an extension:
    the reference's estimate_flow has no such argument) is handed to the
    per-GNC-stage report as compute_flow(init, gt) would get it."""
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
        return ope.compute_flow(np.zeros((H, W, 2)), gt)
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
    fn, flags = progress_printer(ope, gt)  # the reference's compute_flow prints (interface.py:66)
    with ctx.progress(fn, flags):
        ctx.check(ctx.lib.of_estimate_flow(ctx.handle, C.byref(P), nat.ptr(a), nat.ptr(b), H, W, Cc, None,
                                           nat.ptr(out), C.byref(st)))
    ope.alpha = P.alpha
    ope.last_stats = st.as_dict()
    return nat.interleaved(out)


def _as_u8(im):
    a = np.asarray(im)
    if a.dtype == np.uint8:
        return np.ascontiguousarray(a)
    f = np.asarray(a, dtype=float)
    if not (np.all(f == np.floor(f)) and f.min() >= 0 and f.max() <= 255):
        raise ValueError("estimate_flow_batch takes uint8 frames (or integer-valued 0..255)")
    return np.ascontiguousarray(f.astype(np.uint8))


def estimate_flow_batch(im1s, im2s, method='classic+nl-fast', params=None, lanes=4):
    """estimate_flow over a batch of uint8 frame pairs, host to host: one C
    call (of_pairs_run_host) keeps `lanes` pairs in flight on the GPU with
    their uploads and downloads overlapped.  Returns a list of (H, W, 2)
    float64 flows equal to [estimate_flow(a, b, method, params) ...]:
    bitwise with lanes=1 or below 2^20 px; at >= 2^20 px with lanes >= 2 the
    fine CG solves of two pairs run side by side in another block geometry
    and the flows differ by CG rounding only (include/optflow.h)."""
    a = [_as_u8(x) for x in im1s]
    b = [_as_u8(x) for x in im2s]
    if not a or len(a) != len(b):
        raise ValueError("im1s and im2s must be non-empty and of equal length")
    H, W = a[0].shape[:2]
    # every frame of both lists: (H, W) or (H, W, >=3), checked before the
    # [:, :, :3] slice (a 1- or 2-channel frame would otherwise pass as 3)
    for x in a + b:
        if not (x.ndim == 2 or (x.ndim == 3 and x.shape[2] >= 3)):
            raise ValueError("estimate_flow_batch takes (H, W) or (H, W, >=3) frames")
    Cc = 3 if a[0].ndim == 3 else 1
    want = (H, W, 3) if Cc == 3 else (H, W)
    a = [x[:, :, :3] if x.ndim == 3 else x for x in a]
    b = [x[:, :, :3] if x.ndim == 3 else x for x in b]
    for x in a + b:
        if x.shape != want:
            raise ValueError("all frames of a batch must share one shape")
    a = [np.ascontiguousarray(x) for x in a]
    b = [np.ascontiguousarray(x) for x in b]
    ope = load_of_method(method)
    if params is not None:
        ope.parse_input_parameter(params)
    P = ope.to_params()
    P.guide_mode = int(ope._METHOD == 'classic_nl' and ope.color_images is not None)
    n = len(a)
    outs = [np.empty((2, H, W), dtype=np.float32) for _ in range(n)]
    vp = C.c_void_p
    p1 = (vp * n)(*[x.ctypes.data for x in a])
    p2 = (vp * n)(*[x.ctypes.data for x in b])
    po = (vp * n)(*[o.ctypes.data for o in outs])
    ctx = nat.context()
    ctx.check(ctx.lib.of_pairs_run_host(ctx.handle, n, p1, p2, H, W, Cc, C.byref(P), int(lanes), po, None))
    return [nat.interleaved(o) for o in outs]


class PairStream:
    """Streaming estimate_flow over uint8 frame pairs of one shape: a pool of
    `lanes` GPU pipelines (of_pairs_open, include/optflow.h) on a context of
    its own takes pairs as they are submitted, so host work between
    submissions (decoding, writing) never drains the GPU.  Flows equal
    estimate_flow_batch(..., lanes=lanes) bitwise.

        with PairStream(H, W, 3, 'classic+nl-fast') as s:
            t = s.submit(im1, im2)      # returns at once
            uv = s.wait(t)              # (H, W, 2) float64
    """

    def __init__(self, H, W, channels=3, method='classic+nl-fast', params=None, lanes=4, device=0):
        if channels not in (1, 3):
            raise ValueError("channels must be 1 (gray) or 3 (RGB)")
        ope = load_of_method(method)
        if params is not None:
            ope.parse_input_parameter(params)
        P = ope.to_params()
        P.guide_mode = int(ope._METHOD == 'classic_nl' and ope.color_images is not None)
        self.shape = (H, W, 3) if channels == 3 else (H, W)
        self.H, self.W, self.channels = H, W, channels
        self._ctx = nat.Context(device)
        self._live = {}
        try:
            self._ctx.check(self._ctx.lib.of_pairs_open(self._ctx.handle, H, W, channels, C.byref(P), int(lanes)))
        except Exception:
            self._ctx.close()
            raise

    def submit(self, im1, im2):
        """Queue one pair; returns its ticket.  The frames are copied into the
        stream's pinned buffers by a lane thread later, so they are kept
        referenced here until wait()."""
        a = _as_u8(im1)
        b = _as_u8(im2)
        if a.ndim == 3:
            a, b = np.ascontiguousarray(a[:, :, :3]), np.ascontiguousarray(b[:, :, :3])
        if a.shape != self.shape or b.shape != self.shape:
            raise ValueError(f"frames must be {self.shape}, got {a.shape} / {b.shape}")
        out = np.empty((2, self.H, self.W), dtype=np.float32)
        vp = C.c_void_p
        t = C.c_int64(0)
        self._ctx.check(self._ctx.lib.of_pairs_submit(self._ctx.handle, 1, (vp * 1)(a.ctypes.data),
                                                      (vp * 1)(b.ctypes.data), (vp * 1)(out.ctypes.data),
                                                      C.byref(t)))
        self._live[t.value] = (a, b, out)
        return t.value

    def wait(self, ticket, planar=False):
        """Block until the pair's flow is ready; (H, W, 2) float64, or with
        `planar` the library's (2, H, W) float32 planes as they came back (the
        conversion can then run on another thread)."""
        if ticket not in self._live:
            raise ValueError(f"unknown or already waited ticket {ticket}")
        self._ctx.check(self._ctx.lib.of_pairs_wait(self._ctx.handle, int(ticket)))
        out = self._live.pop(ticket)[2]
        return out if planar else nat.interleaved(out)

    def close(self):
        if self._ctx is not None:
            try:
                self._ctx.check(self._ctx.lib.of_pairs_close(self._ctx.handle))
            finally:
                self._ctx.close()
                self._ctx = None
                self._live.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


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
