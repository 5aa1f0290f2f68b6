"""Method registry (reference: optical_flow/methods/config.py:10-176; names,
defaults and overrides reproduced verbatim)."""
import numpy as np

from optical_flow.robust.robust_function import RobustFunction


def load_of_method(method):
    """Return a configured optical-flow object for one of the 12 method names."""
    median_filter_size = [5, 5]

    if method == 'classic+nl-fast':
        ope = load_of_method('classic+nl')
        ope.max_iters = 3
        ope.gnc_iters = 2
        ope.display = True
        return ope

    if method == 'classic+nl':
        from optical_flow.methods.classic_nl import ClassicNLOpticalFlow
        ope = ClassicNLOpticalFlow()
        ope.texture = True
        ope.median_filter_size = median_filter_size
        ope.alp = 0.95
        ope.area_hsz = 7
        ope.sigma_i = 7
        ope.color_images = np.ones((1, 1, 3))
        ope.lambda_ = 3
        ope.lambda_q = 3
        return ope

    if method == 'classic+nl-full':
        ope = load_of_method('classic+nl')
        ope.fullVersion = True
        return ope

    if method == 'hs-brightness':
        from optical_flow.methods.hs import HSOpticalFlow
        ope = HSOpticalFlow()
        ope.median_filter_size = median_filter_size
        ope.lambda_ = 10
        ope.lambda_q = 10
        return ope

    if method == 'hs':
        from optical_flow.methods.hs import HSOpticalFlow
        ope = HSOpticalFlow()
        ope.median_filter_size = median_filter_size
        ope.texture = True
        ope.lambda_ = 40
        ope.lambda_q = 40
        ope.display = True
        return ope

    def _ba(m, s_sp, s_d, lam):
        ope.spatial_filters = [np.array([[1, -1]]), np.array([[1], [-1]])]
        ope.rho_spatial_u = [RobustFunction(m, *s_sp), RobustFunction(m, *s_sp)]
        ope.rho_spatial_v = [RobustFunction(m, *s_sp), RobustFunction(m, *s_sp)]
        ope.rho_data = RobustFunction(m, *s_d)
        ope.lambda_ = lam
        ope.lambda_q = lam

    if method == 'ba-brightness':
        from optical_flow.methods.ba import BAOpticalFlow
        ope = BAOpticalFlow()
        ope.median_filter_size = median_filter_size
        _ba('lorentzian', (0.1,), (3.5,), 0.045)
        return ope

    if method in ('classic-l', 'ba'):
        ope = load_of_method('ba-brightness')
        ope.median_filter_size = median_filter_size
        ope.texture = True
        _ba('lorentzian', (0.03,), (1.5,), 0.06)
        return ope

    if method == 'classic-c-a':
        from optical_flow.methods.alt_ba import AltBAOpticalFlow
        ope = AltBAOpticalFlow()
        ope.median_filter_size = median_filter_size
        ope.texture = True
        _ba('charbonnier', (1e-3,), (1e-3,), 5)
        ope.display = False
        ope.lambda2 = 1e2
        ope.lambda3 = 1
        ope.weightRatio = ope.lambda2 / ope.lambda3
        ope.itersLO = 5
        return ope

    if method == 'classic-c-brightness':
        from optical_flow.methods.ba import BAOpticalFlow
        ope = BAOpticalFlow()
        ope.median_filter_size = median_filter_size
        ope.texture = False
        _ba('charbonnier', (1e-3,), (1e-3,), 3)
        return ope

    if method == 'classic-c':
        ope = load_of_method('classic-c-brightness')
        ope.texture = True
        ope.lambda_ = 5
        ope.lambda_q = 5
        return ope

    if method == 'classic++':
        from optical_flow.methods.ba import BAOpticalFlow
        ope = BAOpticalFlow()
        ope.median_filter_size = median_filter_size
        ope.texture = True
        ope.interpolation_method = 'bi-cubic'
        _ba('generalized_charbonnier', (1e-3, 0.45), (1e-3, 0.45), 3)
        return ope

    raise ValueError(f"Unknown optical flow method: '{method}'")


METHOD_NAMES = ('classic+nl-fast', 'classic+nl', 'classic+nl-full', 'hs-brightness', 'hs', 'ba-brightness',
                'ba', 'classic-l', 'classic-c-a', 'classic-c-brightness', 'classic-c', 'classic++')
