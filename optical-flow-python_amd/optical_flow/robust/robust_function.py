"""RobustFunction: a named penalty plus its parameters
(reference: optical_flow/robust/robust_function.py:16-145)."""
import numpy as np

from optical_flow.robust import penalties as _p

PENALTY_MAP = {
    'quadratic': _p.quadratic,
    'lorentzian': _p.lorentzian,
    'charbonnier': _p.charbonnier,
    'generalized_charbonnier': _p.generalized_charbonnier,
    'geman_mcclure': _p.geman_mcclure,
    'huber': _p.huber,
    'tukey': _p.tukey,
    'gaussian': _p.gaussian,
    'tdist': _p.tdist,
    'tdist_unnorm': _p.tdist_unnorm,
}

_TWO_PARAM = ('generalized_charbonnier', 'tdist', 'tdist_unnorm')


class RobustFunction:
    """Penalty rho with evaluate / deriv / deriv_over_x.

    The GPU kernels read (method, param) from this object when a method's
    attribute bag is flattened into the C ABI's of_params."""

    def __init__(self, method, *args):
        if method not in PENALTY_MAP:
            raise ValueError(f"Unknown penalty method '{method}'. Available: {list(PENALTY_MAP.keys())}")
        self.method = method
        self._func = PENALTY_MAP[method]
        if method in _TWO_PARAM and len(args) >= 2:
            self.sigma = np.array([args[0], args[1]], dtype=float)
        elif len(args) > 0:
            self.sigma = np.atleast_1d(np.asarray(args[0], dtype=float))
        else:
            self.sigma = np.array([1.0])

    @property
    def param(self):
        return self.sigma

    def evaluate(self, x):
        return self._func(np.asarray(x, dtype=float), self.sigma, 0)

    def deriv(self, x):
        return self._func(np.asarray(x, dtype=float), self.sigma, 1)

    def deriv_over_x(self, x):
        return self._func(np.asarray(x, dtype=float), self.sigma, 2)

    def evaluate_log(self, x):
        return self.evaluate(x)

    def __repr__(self):
        return f"RobustFunction('{self.method}', sigma={self.sigma})"
