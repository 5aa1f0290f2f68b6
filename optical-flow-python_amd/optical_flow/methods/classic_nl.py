"""Classic+NL (reference: optical_flow/methods/classic_nl.py:29-378)."""
import numpy as np

from optical_flow import _abi
from optical_flow.methods.base import BaseOpticalFlow
from optical_flow.robust.robust_function import RobustFunction


class ClassicNLOpticalFlow(BaseOpticalFlow):
    """Generalised-Charbonnier IRLS + occlusion-weighted, colour-guided
    weighted median (classic_nl.py:32-87 defaults)."""

    _METHOD = 'classic_nl'

    def __init__(self):
        super().__init__()
        self.lambda_ = 1.0
        self.lambda_q = 1.0
        self.lambda2 = 0.1
        self.lambda3 = 1.0
        self.sor_max_iters = 10000
        self.limit_update = True
        self.display = False
        self.solver = 'backslash'
        self.deriv_filter = np.array([1, -8, 0, 8, -1]) / 12.0
        self.texture = False
        self.fc = False
        self.median_filter_size = None
        self.interpolation_method = 'bi-cubic'
        self.gnc_iters = 3
        self.alpha = 1.0
        self.max_iters = 10
        self.max_linear = 1
        self.pyramid_levels = 4
        self.pyramid_spacing = 2.0
        self.gnc_pyramid_levels = 2
        self.gnc_pyramid_spacing = 1.25
        method = 'generalized_charbonnier'
        a = 0.45
        sig = 1e-3
        self.spatial_filters = [np.array([[1, -1]]), np.array([[1], [-1]])]
        self.rho_spatial_u = [RobustFunction(method, sig, a), RobustFunction(method, sig, a)]
        self.rho_spatial_v = [RobustFunction(method, sig, a), RobustFunction(method, sig, a)]
        self.rho_data = RobustFunction(method, sig, a)
        self.seg = None
        self.mfT = 15
        self.imfsz = [7, 7]
        self.filter_weight = None
        self.alp = 0.95
        self.hybrid = False
        self.area_hsz = 10
        self.affine_hsz = 4
        self.sigma_i = 7
        self.color_images = None
        self.auto_level = True
        self.input_seg = None
        self.input_occ = None
        self.fullVersion = False

    def _qua_penalties(self):
        """classic_nl.py:211-226: quadratic(param[0]) for every penalty."""
        q = lambda r: _abi.penalty('quadratic', float(r.param[0]))  # noqa: E731
        return (q(self.rho_data), [q(r) for r in self.rho_spatial_u], [q(r) for r in self.rho_spatial_v])
