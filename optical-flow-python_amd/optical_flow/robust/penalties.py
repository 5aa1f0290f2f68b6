"""Robust penalty functions rho(x), rho'(x) and rho'(x)/x.

Host-side API utilities with the semantics of the reference's
optical_flow/robust/penalties.py:18-373 (d_type 0 = value, 1 = derivative,
2 = derivative / x, the IRLS weight).  The GPU hot path does not call these:
it evaluates the same weights in-kernel (csrc/common.h: pen_w), checked
against the oracle for every kind in tests/test_gpu_reference_cases.py.
"""
import numpy as np
from scipy.special import gammaln


def _first(sigma):
    return float(np.atleast_1d(sigma)[0])


def _check(d_type):
    if d_type not in (0, 1, 2):
        raise ValueError(f"Unknown d_type: {d_type}")


def quadratic(x, sigma, d_type):
    """x^2 / sigma^2 (penalties.py:18-41)."""
    _check(d_type)
    x = np.asarray(x, dtype=float)
    s2 = _first(sigma) ** 2
    if d_type == 0:
        return x * x / s2
    if d_type == 1:
        return 2.0 * x / s2
    return np.full_like(x, 2.0 / s2)


def lorentzian(x, sigma, d_type):
    """log(1 + x^2 / (2 sigma^2)) (penalties.py:44-67)."""
    _check(d_type)
    x = np.asarray(x, dtype=float)
    s2 = _first(sigma) ** 2
    if d_type == 0:
        return np.log(1.0 + x * x / (2.0 * s2))
    den = 2.0 * s2 + x * x
    return 2.0 * x / den if d_type == 1 else 2.0 / den


def charbonnier(x, sigma, d_type):
    """sig2 * sqrt(1 + (x / sig2)^2) with sig2 = sigma^2 (penalties.py:70-102)."""
    _check(d_type)
    x = np.asarray(x, dtype=float)
    s2 = _first(sigma) ** 2
    root = np.sqrt(1.0 + (x / s2) ** 2)
    if d_type == 0:
        return s2 * root
    return x / (s2 * root) if d_type == 1 else 1.0 / (s2 * root)


def generalized_charbonnier(x, sigma, d_type):
    """(sigma^2 + x^2)^a, sigma = [sig, a] (penalties.py:105-131)."""
    _check(d_type)
    x = np.asarray(x, dtype=float)
    p = np.atleast_1d(sigma)
    sig, a = float(p[0]), float(p[1])
    base = sig * sig + x * x
    if d_type == 0:
        return base ** a
    w = 2.0 * a * base ** (a - 1.0)
    return x * w if d_type == 1 else w


def geman_mcclure(x, sigma, d_type):
    """x^2 / (sigma^2 + x^2) (penalties.py:134-158)."""
    _check(d_type)
    x = np.asarray(x, dtype=float)
    s2 = _first(sigma) ** 2
    den = s2 + x * x
    if d_type == 0:
        return x * x / den
    w = 2.0 * s2 / (den * den)
    return x * w if d_type == 1 else w


def huber(x, sigma, d_type):
    """Quadratic for |x| <= sigma^2, linear beyond (penalties.py:161-198)."""
    _check(d_type)
    x = np.asarray(x, dtype=float)
    s2 = _first(sigma) ** 2
    ax = np.abs(x)
    inl = ax <= s2
    if d_type == 0:
        return np.where(inl, x * x, 2.0 * s2 * ax - s2 * s2)
    if d_type == 1:
        return np.where(inl, 2.0 * x, 2.0 * s2 * np.sign(x))
    return np.where(inl, 2.0, 2.0 * s2 / np.maximum(ax, 1e-30))


def tukey(x, sigma, d_type):
    """Tukey biweight with threshold sigma (penalties.py:201-240)."""
    _check(d_type)
    x = np.asarray(x, dtype=float)
    sig = _first(sigma)
    om = 1.0 - x * x / (sig * sig)
    inl = np.abs(x) <= sig
    if d_type == 0:
        return np.where(inl, (1.0 - om ** 3) / 3.0, 1.0 / 3.0)
    if d_type == 1:
        return np.where(inl, 2.0 * x * om * om / (sig * sig), 0.0)
    return np.where(inl, 2.0 * om * om / (sig * sig), 0.0)


def gaussian(x, sigma, d_type):
    """Gaussian negative log-likelihood (penalties.py:243-268)."""
    _check(d_type)
    x = np.asarray(x, dtype=float)
    sig = _first(sigma)
    if d_type == 0:
        return 0.5 * np.log(2.0 * np.pi) + np.log(sig) + 0.5 * (x / sig) ** 2
    return x / sig ** 2 if d_type == 1 else np.full_like(x, 1.0 / sig ** 2)


def _t(x, sigma, d_type, normalised):
    _check(d_type)
    x = np.asarray(x, dtype=float)
    p = np.atleast_1d(sigma)
    r, s = float(p[0]), float(p[1])
    s2r = s * s * r
    if d_type == 0:
        y = (r + 1.0) / 2.0 * np.log(1.0 + x * x / s2r)
        if normalised:
            y = y + gammaln(r / 2.0) - gammaln((r + 1.0) / 2.0) + 0.5 * np.log(r * np.pi) + np.log(s)
        return y
    w = (r + 1.0) / (s2r + x * x)
    return x * w if d_type == 1 else w


def tdist(x, sigma, d_type):
    """Student-t penalty, sigma = [r, s] (penalties.py:271-313)."""
    return _t(x, sigma, d_type, True)


def tdist_unnorm(x, sigma, d_type):
    """Student-t without the normalising constant (penalties.py:316-345)."""
    return _t(x, sigma, d_type, False)


def mixture(x, sigma, d_type):
    """Not implemented in the reference either (penalties.py:348-361)."""
    raise NotImplementedError("Mixture penalty is not yet implemented.")


def spline_penalty(x, sigma, d_type):
    """Not implemented in the reference either (penalties.py:364-373)."""
    raise NotImplementedError("Spline penalty is not yet implemented.")
