"""Horn-Schunck (reference: optical_flow/methods/hs.py:20-203)."""
import numpy as np

from optical_flow import _abi
from optical_flow.methods.base import BaseOpticalFlow
from optical_flow.robust.robust_function import RobustFunction


class HSOpticalFlow(BaseOpticalFlow):
    """Quadratic data term + Laplacian smoothness (hs.py:23-47 defaults).

    The Laplacian with replicate boundary (hs.py:168-173) equals minus the
    unit-weight 5-point graph Laplacian, so HS runs on the same matrix-free
    operator as BA / Classic+NL with constant weights 1/sigmaD2 (data) and
    lambda/sigmaS2 (edges)."""

    _METHOD = 'hs'

    def __init__(self):
        super().__init__()
        self.lambda_ = 80
        self.lambda_q = 80
        self.gnc_iters = 1
        self.pyramid_levels = 4
        self.pyramid_spacing = 2.0
        self.max_warping_iters = 10
        self.solver = 'backslash'
        self.interpolation_method = 'cubic'
        self.deriv_filter = np.array([1, -8, 0, 8, -1]) / 12.0
        self.texture = False
        self.limit_update = True
        self.display = False
        self.sor_max_iters = 10000
        self.sigmaD2 = 1.0
        self.sigmaS2 = 1.0
        self.mf_iter = 1
        self.color_images = None
        method = 'quadratic'
        self.spatial_filters = [np.array([[1, -1]]), np.array([[1], [-1]])]
        self.rho_spatial_u = [RobustFunction(method, 1), RobustFunction(method, 1)]
        self.rho_spatial_v = [RobustFunction(method, 1), RobustFunction(method, 1)]
        self.rho_data = RobustFunction(method, 1)

    def _robust_penalties(self):
        d = _abi.penalty('const', 1.0 / float(self.sigmaD2))
        s = _abi.penalty('const', 1.0 / float(self.sigmaS2))
        return d, [s, s], [s, s]

    def _qua_penalties(self):
        return self._robust_penalties()

    def _copy_with_images(self, images):
        import copy
        small = copy.copy(self)
        small.images = images
        small.pyramid_levels = 1
        return small

    def flow_operator(self, uv, duv=None, It=None, Ix=None, Iy=None):
        """hs.py:144-203: derivatives are recomputed from self.images."""
        from optical_flow.utils.derivatives import partial_deriv
        It, Ix, Iy = partial_deriv(self.images, uv, self.interpolation_method, self.deriv_filter)
        return super().flow_operator(uv, None, It, Ix, Iy)[0:2] + (None, True)
