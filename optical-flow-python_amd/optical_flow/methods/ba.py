"""Black-Anandan / Classic-C / Classic++ (reference: optical_flow/methods/ba.py:26-302)."""
import numpy as np

from optical_flow import _abi
from optical_flow.methods.base import BaseOpticalFlow
from optical_flow.robust.robust_function import RobustFunction


class BAOpticalFlow(BaseOpticalFlow):
    """Robust data + spatial terms, GNC (ba.py:29-55 defaults)."""

    _METHOD = 'ba'

    def __init__(self):
        super().__init__()
        self.lambda_ = 1.0
        self.lambda_q = 1.0
        self.gnc_iters = 3
        self.alpha = 1.0
        self.max_iters = 10
        self.max_linear = 1
        self.pyramid_levels = 4
        self.pyramid_spacing = 2.0
        self.gnc_pyramid_levels = 2
        self.gnc_pyramid_spacing = 1.25
        self.texture = False
        self.fc = False
        self.blend = 0.5
        self.alp = 0.95
        self.auto_level = True
        self.solver = 'backslash'
        self.interpolation_method = 'cubic'
        self.deriv_filter = np.array([1, -8, 0, 8, -1]) / 12.0
        self.limit_update = True
        self.display = False
        self.sor_max_iters = 10000
        self.color_images = None
        method = 'lorentzian'
        self.spatial_filters = [np.array([[1, -1]]), np.array([[1], [-1]])]
        self.rho_spatial_u = [RobustFunction(method, 0.03), RobustFunction(method, 0.03)]
        self.rho_spatial_v = [RobustFunction(method, 0.03), RobustFunction(method, 0.03)]
        self.rho_data = RobustFunction(method, 1.5)

    def _qua_penalties(self):
        """ba.py:152-163: quadratic(1) spatial, quadratic(sigma_d / sigma_s) data."""
        ta = float(self.rho_data.param[0]) / float(self.rho_spatial_u[0].param[0])
        one = _abi.penalty('quadratic', 1.0)
        return (_abi.penalty('quadratic', ta), [one for _ in self.rho_spatial_u],
                [one for _ in self.rho_spatial_v])
