"""The reference-side binding: the file a maintainer of
jordanshivers/optical-flow-python drops into the reference package as
`optical_flow/_mi355x.py` to route `estimate_flow` (interface.py:11-71) to
liboptflow.so through ctypes.

It depends on nothing from this repository: numpy, ctypes, its own mirror of
`of_params` (include/optflow.h, ABI 3), and — only inside `estimate_flow` —
the host package's `optical_flow.methods.config.load_of_method`, which inside
the reference is the reference's own registry (config.py:10-176).
`of_params_from(ope)` reads only attributes the reference's classes define:

    BaseOpticalFlow.__init__         base.py:21-63
    ClassicNLOpticalFlow.__init__    classic_nl.py:32-87
    BAOpticalFlow.__init__           ba.py:26-55
    HSOpticalFlow.__init__           hs.py:23-47
    AltBAOpticalFlow.__init__        alt_ba.py:31-79
    RobustFunction.method / .sigma   robust_function.py:65-83

and picks the method kind (and the colour guide of the weighted median) from
the class name.  The GPU-only knobs of the 'backslash' surrogate (SuperLU,
base.py:107-108, is replaced by block-Jacobi PCG to a 1e-6 true residual) are
module constants here, since the reference has no attribute for them.

Hook in the reference's interface.py, first line of estimate_flow():

    if os.environ.get("OPTFLOW_BACKEND") == "mi355x":
        from optical_flow._mi355x import estimate_flow as _gpu
        return _gpu(im1, im2, method, params)

tests/test_reference_hook.py pins of_params_from against this repository's
own to_params() on the reference's attribute bags (tests/golden/ref_bags.json,
written by gen_golden.py by importing the reference), against the live
reference when it is importable, and (-m gpu) runs estimate_flow through the
C ABI on the golden crop.
"""
import ctypes as C
import ctypes.util
import os

import numpy as np

OF_ABI_VERSION = 3
OF_EINVAL, OF_ENOTSUP = -1, -4

# 'backslash' surrogate (no reference attribute): PCG relative-residual target
# and iteration cap
BACKSLASH_RTOL = 1e-6
BACKSLASH_MAXITER = 2000

_METHOD_OF_CLASS = {"HSOpticalFlow": 0, "BAOpticalFlow": 1, "ClassicNLOpticalFlow": 2, "AltBAOpticalFlow": 3}
_INTERP = {"cubic": 0, "bi-cubic": 1, "bi-linear": 2}
_SOLVER = {"backslash": 0, "pcg": 1, "sor": 2}
_PENALTY = {"quadratic": 0, "lorentzian": 1, "charbonnier": 2, "generalized_charbonnier": 3,
            "geman_mcclure": 4, "huber": 5, "tukey": 6, "gaussian": 7, "tdist": 8, "tdist_unnorm": 9}
_PEN_CONST = 100
_MAX_FILTERS, _MAX_FDIM = 8, 5


class _Penalty(C.Structure):
    _fields_ = [("kind", C.c_int32), ("pad_", C.c_int32), ("p0", C.c_double), ("p1", C.c_double)]


class _FilterSet(C.Structure):
    _fields_ = [("general", C.c_int32), ("n", C.c_int32),
                ("fh", C.c_int32 * _MAX_FILTERS), ("fw", C.c_int32 * _MAX_FILTERS),
                ("taps", (C.c_double * (_MAX_FDIM * _MAX_FDIM)) * _MAX_FILTERS),
                ("rho_u", _Penalty * _MAX_FILTERS), ("rho_v", _Penalty * _MAX_FILTERS),
                ("qua_u", _Penalty * _MAX_FILTERS), ("qua_v", _Penalty * _MAX_FILTERS)]


class OfParams(C.Structure):
    """of_params (include/optflow.h:93-137)."""
    _fields_ = ([(n, C.c_int32) for n in (
        "method", "solver", "interp", "texture", "fc", "auto_level", "pyramid_levels", "gnc_iters",
        "gnc_pyramid_levels", "max_iters", "max_warping_iters", "max_linear", "pcg_maxiter",
        "sor_max_iters", "limit_update", "median_filter_size", "mf_iter", "use_wmf", "area_hsz",
        "itersLO", "exact_maxiter", "display", "guide_mode", "pad_")]
        + [(n, C.c_double) for n in (
            "lambda_", "lambda_q", "alpha", "pyramid_spacing", "gnc_pyramid_spacing", "pcg_rtol",
            "exact_rtol", "sor_omega", "sor_tol", "blend", "alp", "sigma_i", "sigmaD2", "sigmaS2",
            "lambda2", "lambda3")]
        + [("deriv_filter", C.c_double * 5),
           ("rho_data", _Penalty), ("rho_spatial_u", _Penalty * 2), ("rho_spatial_v", _Penalty * 2),
           ("qua_data", _Penalty), ("qua_spatial_u", _Penalty * 2), ("qua_spatial_v", _Penalty * 2),
           ("rho_couple", _Penalty), ("filters", _FilterSet)])


# ---------------------------------------------------------------------------
# attribute bag -> of_params
# ---------------------------------------------------------------------------
def method_kind(ope):
    """of_method from the class (or the first known base class) name."""
    for cls in type(ope).__mro__:
        if cls.__name__ in _METHOD_OF_CLASS:
            return _METHOD_OF_CLASS[cls.__name__]
    raise ValueError(f"not an optical-flow method object: {type(ope).__name__}")


def _pen(rf):
    """RobustFunction(method, *args) -> of_penalty: .sigma holds [sigma] or
    [sigma, a] / [r, s] (robust_function.py:65-83)."""
    if rf.method not in _PENALTY:
        raise ValueError(f"Unknown penalty method '{rf.method}'")
    s = np.atleast_1d(np.asarray(rf.sigma, dtype=float))
    return _Penalty(_PENALTY[rf.method], 0, float(s[0]), float(s[1]) if s.size > 1 else 0.0)


def _quadratic(p0):
    return _Penalty(_PENALTY["quadratic"], 0, float(p0), 0.0)


def _const(p0):
    return _Penalty(_PEN_CONST, 0, float(p0), 0.0)


def _penalties(ope, kind):
    """(rho_data, rho_u, rho_v) and their quadratic relaxations (qua_*), as
    compute_flow_base builds them per class."""
    su, sv = list(ope.rho_spatial_u), list(ope.rho_spatial_v)
    if kind == 0:
        # hs.py:195-201: data / sigmaD2, Laplacian / sigmaS2, no penalties
        d, s = _const(1.0 / float(ope.sigmaD2)), _const(1.0 / float(ope.sigmaS2))
        rho = (d, [s, s], [s, s])
        return rho, rho
    rho = (_pen(ope.rho_data), [_pen(r) for r in su], [_pen(r) for r in sv])
    if kind == 2:
        # classic_nl.py:211-226: quadratic(param[0]) for every penalty
        first = lambda r: float(np.atleast_1d(r.sigma)[0])  # noqa: E731
        qua = (_quadratic(first(ope.rho_data)), [_quadratic(first(r)) for r in su],
               [_quadratic(first(r)) for r in sv])
    elif kind == 1:
        # ba.py:152-163: quadratic(1) spatial, quadratic(sigma_d / sigma_s) data
        ta = float(np.atleast_1d(ope.rho_data.sigma)[0]) / float(np.atleast_1d(su[0].sigma)[0])
        qua = (_quadratic(ta), [_quadratic(1.0) for _ in su], [_quadratic(1.0) for _ in sv])
    else:
        # alt_ba.py:201-207: quadratic(1) everywhere
        qua = (_quadratic(1.0), [_quadratic(1.0) for _ in su], [_quadratic(1.0) for _ in sv])
    return rho, qua


def _median_size(mfsz):
    if mfsz is None:
        return 0
    s = (int(mfsz), int(mfsz)) if np.ndim(mfsz) == 0 else tuple(int(v) for v in mfsz)
    if len(s) != 2 or s[0] != s[1] or s[0] % 2 == 0:
        raise NotImplementedError(f"median_filter_size must be an odd square size, got {mfsz}")
    return s[0]


_DEFAULT_PAIR = (np.array([[1, -1]]), np.array([[1], [-1]]))


def _general_filters(ope, kind):
    if kind == 0:  # HS assembles its own Laplacian (hs.py:168-173)
        return None
    fs = [np.atleast_2d(np.asarray(f, dtype=float)) for f in ope.spatial_filters]
    if len(fs) == 2 and all(f.shape == d.shape and np.array_equal(f, d) for f, d in zip(fs, _DEFAULT_PAIR)):
        return None
    if len(fs) > _MAX_FILTERS or any(f.ndim != 2 or max(f.shape) > _MAX_FDIM for f in fs):
        raise NotImplementedError(f"at most {_MAX_FILTERS} spatial filters of at most {_MAX_FDIM}x{_MAX_FDIM} taps")
    return fs


def of_params_from(ope, backslash_rtol=BACKSLASH_RTOL, backslash_maxiter=BACKSLASH_MAXITER):
    """Flatten a reference method object's attribute bag into of_params.

    Attributes a class does not define take that class's effective default
    (e.g. `max_warping_iters` exists on HS only, `area_hsz` / `sigma_i` on
    Classic+NL only, `lambda2` on Classic+NL / AltBA only)."""
    kind = method_kind(ope)
    g = lambda name, dflt: getattr(ope, name, dflt)  # noqa: E731
    P = OfParams()
    P.method = kind
    solver = str(ope.solver).lower()
    if solver not in _SOLVER:
        raise ValueError(f"Unknown solver: {ope.solver}")
    P.solver = _SOLVER[solver]
    if ope.interpolation_method not in _INTERP:
        raise ValueError(f"Unknown interpolation method: {ope.interpolation_method}")
    P.interp = _INTERP[ope.interpolation_method]
    P.texture = int(bool(ope.texture))
    P.fc = int(bool(g("fc", False)))
    P.auto_level = int(bool(g("auto_level", True)))
    P.pyramid_levels = int(ope.pyramid_levels)
    P.gnc_iters = int(ope.gnc_iters)
    P.gnc_pyramid_levels = int(ope.gnc_pyramid_levels)
    P.max_iters = int(ope.max_iters)
    P.max_warping_iters = int(g("max_warping_iters", 10))
    P.max_linear = int(ope.max_linear)
    P.pcg_maxiter = int(ope.pcg_maxiter)
    P.sor_max_iters = int(ope.sor_max_iters)
    P.limit_update = int(bool(ope.limit_update))
    P.median_filter_size = _median_size(ope.median_filter_size)
    P.mf_iter = int(g("mf_iter", 1))
    P.use_wmf = int(kind == 2 and P.median_filter_size > 0)
    P.area_hsz = int(g("area_hsz", 7))
    P.itersLO = int(g("itersLO", 1))
    P.exact_maxiter = int(backslash_maxiter)
    P.display = int(bool(ope.display))
    P.guide_mode = int(kind == 2 and ope.color_images is not None)
    P.lambda_ = float(ope.lambda_)
    P.lambda_q = float(ope.lambda_q)
    P.alpha = float(ope.alpha)
    P.pyramid_spacing = float(ope.pyramid_spacing)
    P.gnc_pyramid_spacing = float(ope.gnc_pyramid_spacing)
    P.pcg_rtol = float(ope.pcg_rtol)
    P.exact_rtol = float(backslash_rtol)
    P.sor_omega = 1.9   # base.py:109
    P.sor_tol = 1e-2    # base.py:109
    P.blend = float(ope.blend)
    P.alp = float(ope.alp)
    P.sigma_i = float(g("sigma_i", 7.0))
    P.sigmaD2 = float(g("sigmaD2", 1.0))
    P.sigmaS2 = float(g("sigmaS2", 1.0))
    P.lambda2 = float(g("lambda2", 0.0))
    P.lambda3 = float(g("lambda3", 1.0))
    df = np.asarray(ope.deriv_filter, dtype=float).ravel()
    if df.size != 5:
        raise NotImplementedError("deriv_filter must have 5 taps")
    for k, v in enumerate(df):
        P.deriv_filter[k] = v
    fs = _general_filters(ope, kind)
    nf = 2 if fs is None else len(fs)
    if len(ope.rho_spatial_u) < nf or len(ope.rho_spatial_v) < nf:
        # the reference indexes rho_spatial_u[i] per filter (classic_nl.py:315-316)
        raise IndexError("rho_spatial_u / rho_spatial_v need one penalty per spatial filter")
    (d, su, sv), (qd, qsu, qsv) = _penalties(ope, kind)
    P.rho_data, P.qua_data = d, qd
    for k in range(min(2, len(su))):
        P.rho_spatial_u[k], P.qua_spatial_u[k] = su[k], qsu[k]
    for k in range(min(2, len(sv))):
        P.rho_spatial_v[k], P.qua_spatial_v[k] = sv[k], qsv[k]
    if fs is not None:
        F = P.filters
        F.general, F.n = 1, len(fs)
        for q, f in enumerate(fs):
            F.fh[q], F.fw[q] = f.shape
            for t, v in enumerate(f.ravel()):
                F.taps[q][t] = float(v)
            F.rho_u[q], F.rho_v[q], F.qua_u[q], F.qua_v[q] = su[q], sv[q], qsu[q], qsv[q]
    rc = g("rho_couple", None)
    P.rho_couple = _pen(rc) if rc is not None else _Penalty(_PENALTY["charbonnier"], 0, 1e-3, 0.0)
    return P


# ---------------------------------------------------------------------------
# library + estimate_flow
# ---------------------------------------------------------------------------
_fp = C.POINTER(C.c_float)
_LIB = None


def load_lib(path=None):
    """liboptflow.so: `path`, $OPTFLOW_LIB, the loader's search path, or this
    repository's in-tree build (when run from tools/)."""
    global _LIB
    if path is None and _LIB is not None:
        return _LIB
    cands = [path, os.environ.get("OPTFLOW_LIB"), ctypes.util.find_library("optflow"),
             os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                          "optical-flow-python_amd", "optical_flow", "_lib", "liboptflow.so")]
    p = next((c for c in cands if c and (os.path.exists(c) or not os.path.isabs(c))), None)
    if p is None:
        raise RuntimeError("liboptflow.so not found (set OPTFLOW_LIB)")
    lib = C.CDLL(p)
    lib.of_last_error.restype = C.c_char_p
    lib.of_last_error.argtypes = [C.c_void_p]
    if lib.of_abi_version() != OF_ABI_VERSION:
        raise RuntimeError("liboptflow.so ABI version mismatch")
    if path is None:
        _LIB = lib
    return lib


def _check(lib, ctx, rc):
    if rc != 0:
        msg = (lib.of_last_error(ctx) or b"").decode()
        raise (ValueError if rc == OF_EINVAL else NotImplementedError if rc == OF_ENOTSUP else RuntimeError)(msg)


def _planar(a):
    a = np.asarray(a, dtype=np.float32)
    return np.ascontiguousarray(np.moveaxis(a, 2, 0) if a.ndim == 3 else a)


def estimate_flow_ope(ope, im1, im2, lib=None):
    """The body of estimate_flow (interface.py:35-71) for a configured method
    object: RGB -> gray / Lab on the device, then compute_flow with a zero
    initial flow.  Returns (H, W, 2) float64; `ope` is not modified."""
    lib = lib or load_lib()
    im1 = np.asarray(im1, dtype=float)
    im2 = np.asarray(im2, dtype=float)
    if im1.shape != im2.shape or im1.ndim not in (2, 3):
        raise ValueError("im1 and im2 must be (H, W) or (H, W, C) of one shape")
    P = of_params_from(ope)
    H, W = im1.shape[:2]
    out = np.empty((2, H, W), np.float32)
    ctx = C.c_void_p()
    _check(lib, None, lib.of_ctx_create(0, C.byref(ctx)))
    try:
        if im1.ndim == 3 and im1.shape[2] < 3:
            # interface.py:47 + 62-63: channels concatenated, guide = im1
            nc = im1.shape[2]
            images = _planar(np.concatenate([im1, im2], axis=2))
            guide = _planar(im1) if P.guide_mode else None
            _check(lib, ctx, lib.of_compute_flow(ctx, C.byref(P), images.ctypes.data_as(_fp), H, W, nc,
                                                 None if guide is None else guide.ctypes.data_as(_fp),
                                                 nc if guide is not None else 0, None,
                                                 out.ctypes.data_as(_fp), None))
        else:
            cn = 3 if im1.ndim == 3 else 1
            a = np.ascontiguousarray(im1[..., :3] if cn == 3 else im1, np.float32)
            b = np.ascontiguousarray(im2[..., :3] if cn == 3 else im2, np.float32)
            _check(lib, ctx, lib.of_estimate_flow(ctx, C.byref(P), a.ctypes.data_as(_fp), b.ctypes.data_as(_fp),
                                                  H, W, cn, None, out.ctypes.data_as(_fp), None))
    finally:
        lib.of_ctx_destroy(ctx)
    return np.moveaxis(out, 0, 2).astype(np.float64)


def estimate_flow(im1, im2, method="classic+nl-fast", params=None, lib=None):
    """interface.py:11-71 on the GPU: the host package's registry and
    parse_input_parameter (base.py:65-85: 'lambda' -> lambda_, unknown keys
    ignored, dict or flat [key, val, ...]), then estimate_flow_ope."""
    from optical_flow.methods.config import load_of_method
    ope = load_of_method(method)  # ValueError on an unknown name (config.py:174-176)
    if params is not None:
        ope.parse_input_parameter(params)
    return estimate_flow_ope(ope, im1, im2, lib)
