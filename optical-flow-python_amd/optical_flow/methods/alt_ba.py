"""Alternative BA with auxiliary flow + Li-Osher median
(reference: optical_flow/methods/alt_ba.py:28-372)."""
import ctypes as C

import numpy as np

from optical_flow import _abi
from optical_flow import _native as nat
from optical_flow.methods.base import BaseOpticalFlow, progress_printer
from optical_flow.robust.robust_function import RobustFunction


class AltBAOpticalFlow(BaseOpticalFlow):
    """alt_ba.py:31-79 defaults.  compute_flow returns uvhat (alt_ba.py:185-187)."""

    _METHOD = 'alt_ba'

    def __init__(self):
        super().__init__()
        self.lambda_ = 5.0
        self.lambda_q = 5.0
        self.sor_max_iters = 10000
        self.limit_update = True
        self.display = False
        self.solver = 'backslash'
        self.warping_mode = 'backward'
        self.texture = False
        self.deriv_filter = np.array([1, -8, 0, 8, -1]) / 12.0
        self.median_filter_size = None
        self.interpolation_method = 'cubic'
        self.gnc_iters = 3
        self.alpha = 1.0
        self.max_iters = 10
        self.max_linear = 1
        self.pyramid_levels = 4
        self.pyramid_spacing = 2.0
        self.gnc_pyramid_levels = 2
        self.gnc_pyramid_spacing = 1.25
        method = 'lorentzian'
        self.spatial_filters = [np.array([[1, -1]]), np.array([[1], [-1]])]
        self.rho_spatial_u = [RobustFunction(method, 0.03), RobustFunction(method, 0.03)]
        self.rho_spatial_v = [RobustFunction(method, 0.03), RobustFunction(method, 0.03)]
        self.rho_data = RobustFunction(method, 1.5)
        self.seg = None
        self.mfT = 15
        self.imfsz = [7, 7]
        self.qterm = True
        self.lambda2 = 0.1
        self.lambda3 = 1.0
        self.weightRatio = 1.0
        self.itersLO = 1
        self.color_images = None
        self.replacement = True
        self.rho_couple = RobustFunction('charbonnier', 1e-3)
        self.auto_level = True

    def _qua_penalties(self):
        """alt_ba.py:201-207: quadratic(1) everywhere."""
        one = _abi.penalty('quadratic', 1.0)
        return one, [one for _ in self.rho_spatial_u], [one for _ in self.rho_spatial_v]

    def compute_flow_base(self, uv, uvhat):
        """One pyramid level with coupling and Li-Osher denoising
        (alt_ba.py:189-274) on self.images with self.alpha and
        self.replacement; returns (uv, uvhat)."""
        images, H, W, nc = self._images_planar()
        P = self.to_params()
        out_uv = np.empty((2, H, W), dtype=np.float32)
        out_hat = np.empty((2, H, W), dtype=np.float32)
        ctx = nat.context()
        fn, flags = progress_printer(self, None)
        with ctx.progress(fn, flags):
            ctx.check(ctx.lib.of_alt_ba_flow_base(ctx.handle, C.byref(P), nat.ptr(images), H, W, nc,
                                                  float(self.alpha), int(bool(self.replacement)),
                                                  nat.ptr(nat.planar(uv)), nat.ptr(nat.planar(uvhat)),
                                                  nat.ptr(out_uv), nat.ptr(out_hat)))
        return nat.interleaved(out_uv), nat.interleaved(out_hat)
