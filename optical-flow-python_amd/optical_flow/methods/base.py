"""BaseOpticalFlow: the attribute bag + the seam to the GPU library.

Mirrors optical_flow/methods/base.py:18-281 of the reference: same attribute
names and defaults, same parse_input_parameter semantics, same public methods.
compute_flow / compute_flow_base / flow_operator / _solve_linear_system run
on the GPU through liboptflow.so (include/optflow.h); there is no CPU path.
"""
import ctypes as C
from abc import ABC

import numpy as np
from scipy import sparse

from optical_flow import _abi
from optical_flow import _native as nat
from optical_flow.robust.robust_function import RobustFunction

_DEFAULT_FILTERS = (np.array([[1, -1]]), np.array([[1], [-1]]))


def progress_printer(ope, gt):
    """(callback, of_set_progress flags) printing what the reference's
    compute_flow prints for `ope`: with ope.display the GNC stage / pyramid
    level headers and each iteration's ||x - duv|| (HS: ||x||)
    (classic_nl.py:141-152, 255-256; ba.py:101-114, 189-190; hs.py:80-81,
    123-124; alt_ba.py:128-139, 249-250), and after every GNC stage (always,
    not for HS) "GNC stage k finished, m minutes passed", with `gt` the
    stage's AAE / STD / EPE (classic_nl.py:186-196; alt_ba.py:175-183 prints
    them on a line of their own; ba.py:132-133 has none)."""
    meth = ope._METHOD
    display = bool(getattr(ope, 'display', False))
    want_flow = gt is not None and meth in ('classic_nl', 'alt_ba')
    flags = (_abi.OF_PROGRESS_ITER if display else 0) | (_abi.OF_PROGRESS_FLOW if want_flow else 0)

    def fn(e):
        if e.event == _abi.OF_EV_STAGE:
            if display and meth != 'hs':
                print(f"GNC stage: {e.stage + 1}")
        elif e.event == _abi.OF_EV_LEVEL:
            if display:
                print(f"Pyramid level: {e.level + 1}" if meth == 'hs' else f"  Pyramid level: {e.level + 1}")
        elif e.event == _abi.OF_EV_ITER:
            if display:
                if meth == 'hs':
                    print(f"  Iteration: {e.iter + 1}  (norm: {e.norm:.6f})")
                else:
                    print(f"    Iter: {e.iter + 1} {e.lin + 1} (delta: {e.norm:.6f})")
        elif e.event == _abi.OF_EV_STAGE_END and meth != 'hs':
            msg = f"GNC stage {e.stage + 1} finished, {e.elapsed_s / 60:.2f} minutes passed"
            extra = None
            if want_flow and e.uv:
                from optical_flow.evaluation.metrics import flow_angular_error
                uv = np.ctypeslib.as_array(e.uv, shape=(2, e.h, e.w)).astype(np.float64)
                g = np.asarray(gt, dtype=float)
                if g.shape[:2] == (e.h, e.w):
                    aae, stdae, aepe = flow_angular_error(g[:, :, 0], g[:, :, 1], uv[0], uv[1], 0)
                    extra = f"AAE {aae:.3f} STD {stdae:.3f} EPE {aepe:.3f}"
            if extra and meth == 'classic_nl':
                msg += "  " + extra
            print(msg)
            if extra and meth == 'alt_ba':
                print("  " + extra)
    return fn, flags


class BaseOpticalFlow(ABC):
    """Base class for variational optical flow estimation (base.py:18-63)."""

    _METHOD = None  # one of _abi.METHOD

    def __init__(self):
        self.images = None
        self.lambda_ = 1.0
        self.lambda_q = 1.0
        self.solver = 'backslash'
        self.pcg_rtol = 1e-3
        self.pcg_maxiter = 200
        self.sor_max_iters = 10000
        self.interpolation_method = 'cubic'
        self.deriv_filter = np.array([1, -8, 0, 8, -1]) / 12.0
        self.blend = 0.5
        self.texture = False
        self.fc = False
        self.median_filter_size = None
        self.limit_update = True
        self.display = False
        self.color_images = None
        self.auto_level = True
        self.alp = 0.95
        self.pyramid_levels = 4
        self.pyramid_spacing = 2.0
        self.gnc_iters = 1
        self.gnc_pyramid_levels = 2
        self.gnc_pyramid_spacing = 1.25
        self.alpha = 1.0
        self.max_iters = 10
        self.max_linear = 1
        self.spatial_filters = [np.array([[1, -1]]), np.array([[1], [-1]])]
        method = 'quadratic'
        self.rho_spatial_u = [RobustFunction(method, 1), RobustFunction(method, 1)]
        self.rho_spatial_v = [RobustFunction(method, 1), RobustFunction(method, 1)]
        self.rho_data = RobustFunction(method, 1)
        # GPU 'backslash' surrogate: the reference's direct SuperLU solve is
        # replaced by a 2x2-block-Jacobi PCG run to this relative residual
        # ("Solver parity").
        self.backslash_rtol = 1e-6
        self.backslash_maxiter = 2000
        self.last_stats = None

    # ---- reference API -------------------------------------------------
    def parse_input_parameter(self, params):
        """dict or MATLAB-style flat [key, val, ...]; 'lambda' -> lambda_;
        unknown keys are ignored (base.py:65-85)."""
        if isinstance(params, dict):
            items = list(params.items())
        elif isinstance(params, (list, tuple)):
            items = [(params[i], params[i + 1]) for i in range(0, len(params) - 1, 2)]
        else:
            return
        for key, val in items:
            attr = 'lambda_' if key == 'lambda' else key
            if hasattr(self, attr):
                setattr(self, attr, val)

    def _auto_pyramid_levels(self, images):
        """base.py:192-195."""
        min_dim = min(images.shape[0], images.shape[1])
        return 1 + int(np.floor(np.log(min_dim / 16.0) / np.log(self.pyramid_spacing)))

    def _build_pyramid(self, images, levels, spacing):
        """base.py:174-190, on the GPU."""
        from optical_flow.utils.pyramid import compute_image_pyramid
        from optical_flow.utils.image_processing import fspecial_gaussian
        sigma = np.sqrt(spacing) / np.sqrt(2)
        ksize = 2 * round(1.5 * sigma) + 1
        return compute_image_pyramid(images, fspecial_gaussian(int(ksize), sigma), levels, 1.0 / spacing)

    def clear_conv_cache(self):
        """No sparse matrices are cached: the operator is matrix-free."""

    # ---- parameter flattening -------------------------------------------
    def _robust_penalties(self):
        return (_abi.penalty_from_robust(self.rho_data),
                [_abi.penalty_from_robust(r) for r in self.rho_spatial_u],
                [_abi.penalty_from_robust(r) for r in self.rho_spatial_v])

    def _qua_penalties(self):
        raise NotImplementedError

    def _general_filters(self):
        """True when spatial_filters is not the default [[1, -1]], [[1], [-1]]
        pair (the 5-point hot path); HS never uses spatial_filters (hs.py
        assembles its own Laplacian)."""
        if self._METHOD == 'hs':
            return False
        return len(self.spatial_filters) != 2 or any(
            np.asarray(f).shape != d.shape or not np.array_equal(np.asarray(f), d)
            for f, d in zip(self.spatial_filters, _DEFAULT_FILTERS))

    def _check_supported(self):
        if self._general_filters():
            if len(self.spatial_filters) > _abi.MAX_FILTERS:
                raise NotImplementedError(f"at most {_abi.MAX_FILTERS} spatial_filters are supported")
            for f in self.spatial_filters:
                f = np.atleast_2d(np.asarray(f, dtype=float))
                if f.ndim != 2 or f.shape[0] > _abi.MAX_FDIM or f.shape[1] > _abi.MAX_FDIM:
                    raise NotImplementedError(f"spatial filters of at most {_abi.MAX_FDIM} x {_abi.MAX_FDIM} taps")
            if len(self.rho_spatial_u) < len(self.spatial_filters) or \
                    len(self.rho_spatial_v) < len(self.spatial_filters):
                # the reference indexes rho_spatial_u[i] per filter (classic_nl.py:315-316)
                raise IndexError("rho_spatial_u / rho_spatial_v need one penalty per spatial filter")
        elif len(self.rho_spatial_u) < 2 or len(self.rho_spatial_v) < 2:
            raise IndexError("rho_spatial_u / rho_spatial_v need one penalty per spatial filter")
        if np.asarray(self.deriv_filter).size != 5:
            raise NotImplementedError("deriv_filter must have 5 taps")

    @staticmethod
    def _mf_size(mfsz):
        if mfsz is None:
            return 0
        if np.ndim(mfsz) == 0:
            s = (int(mfsz), int(mfsz))
        else:
            s = tuple(int(v) for v in mfsz)
        if len(s) != 2 or s[0] != s[1] or s[0] % 2 == 0:
            raise NotImplementedError(f"median_filter_size must be an odd square size, got {mfsz}")
        return s[0]

    def to_params(self):
        """Flatten the attribute bag into the C ABI's of_params."""
        self._check_supported()
        P = _abi.OfParams()
        P.method = _abi.METHOD[self._METHOD]
        solver = str(self.solver).lower()
        if solver not in _abi.SOLVER:
            raise ValueError(f"Unknown solver: {self.solver}")
        P.solver = _abi.SOLVER[solver]
        if self.interpolation_method not in _abi.INTERP:
            raise ValueError(f"Unknown interpolation method: {self.interpolation_method}")
        P.interp = _abi.INTERP[self.interpolation_method]
        P.texture = int(bool(self.texture))
        P.fc = int(bool(getattr(self, 'fc', False)))
        P.auto_level = int(bool(getattr(self, 'auto_level', True)))
        P.pyramid_levels = int(self.pyramid_levels)
        P.gnc_iters = int(self.gnc_iters)
        P.gnc_pyramid_levels = int(self.gnc_pyramid_levels)
        P.max_iters = int(self.max_iters)
        P.max_warping_iters = int(getattr(self, 'max_warping_iters', 10))
        P.max_linear = int(self.max_linear)
        P.pcg_maxiter = int(self.pcg_maxiter)
        P.sor_max_iters = int(self.sor_max_iters)
        P.limit_update = int(bool(self.limit_update))
        P.median_filter_size = self._mf_size(self.median_filter_size)
        P.mf_iter = int(getattr(self, 'mf_iter', 1))
        P.use_wmf = int(self._METHOD == 'classic_nl' and P.median_filter_size > 0)
        P.area_hsz = int(getattr(self, 'area_hsz', 7))
        P.itersLO = int(getattr(self, 'itersLO', 1))
        P.exact_maxiter = int(self.backslash_maxiter)
        P.display = int(bool(self.display))
        P.guide_mode = int(self._METHOD == 'classic_nl' and self.color_images is not None)
        P.lambda_ = float(self.lambda_)
        P.lambda_q = float(self.lambda_q)
        P.alpha = float(self.alpha)
        P.pyramid_spacing = float(self.pyramid_spacing)
        P.gnc_pyramid_spacing = float(self.gnc_pyramid_spacing)
        P.pcg_rtol = float(self.pcg_rtol)
        P.exact_rtol = float(self.backslash_rtol)
        P.sor_omega = 1.9   # base.py:109
        P.sor_tol = 1e-2    # base.py:109
        P.blend = float(self.blend)
        P.alp = float(self.alp)
        P.sigma_i = float(getattr(self, 'sigma_i', 7.0))
        P.sigmaD2 = float(getattr(self, 'sigmaD2', 1.0))
        P.sigmaS2 = float(getattr(self, 'sigmaS2', 1.0))
        P.lambda2 = float(getattr(self, 'lambda2', 0.0))
        P.lambda3 = float(getattr(self, 'lambda3', 1.0))
        for k, v in enumerate(np.asarray(self.deriv_filter, dtype=float).ravel()):
            P.deriv_filter[k] = v
        d, su, sv = self._robust_penalties()
        qd, qsu, qsv = self._qua_penalties()
        P.rho_data = d
        P.qua_data = qd
        # default-pair slots; a general filter list may carry fewer penalties
        # per component (each list guarded on its own length)
        for k in range(min(2, len(su))):
            P.rho_spatial_u[k], P.qua_spatial_u[k] = su[k], qsu[k]
        for k in range(min(2, len(sv))):
            P.rho_spatial_v[k], P.qua_spatial_v[k] = sv[k], qsv[k]
        if self._general_filters():
            F = P.filters
            F.general = 1
            F.n = len(self.spatial_filters)
            for q, f in enumerate(self.spatial_filters):
                f = np.atleast_2d(np.asarray(f, dtype=float))
                F.fh[q], F.fw[q] = f.shape
                for t, v in enumerate(f.ravel()):
                    F.taps[q][t] = float(v)
                F.rho_u[q], F.rho_v[q] = su[q], sv[q]
                F.qua_u[q], F.qua_v[q] = qsu[q], qsv[q]
        rc = getattr(self, 'rho_couple', None)
        P.rho_couple = _abi.penalty_from_robust(rc) if rc is not None else _abi.penalty('charbonnier', 1e-3)
        return P

    # ---- GPU seam --------------------------------------------------------
    def _images_planar(self):
        if self.images is None:
            raise ValueError("images not set")
        im = np.asarray(self.images, dtype=float)
        if im.ndim != 3 or im.shape[2] % 2:
            raise ValueError(f"images must be (H, W, 2*nc), got {im.shape}")
        return nat.planar(im), im.shape[0], im.shape[1], im.shape[2] // 2

    def _guide_planar(self, H, W):
        """color_images handling of weighted_median.py:42-59."""
        if self._METHOD != 'classic_nl' or self.color_images is None:
            return None, 0
        g = np.asarray(self.color_images, dtype=float)
        if g.shape[0] != H or g.shape[1] != W:
            if g.size < H * W:
                return None, 0  # reference falls back to a plain median
            raise NotImplementedError("colour guide of a different size (skimage resize path)")
        g = nat.planar(g)
        return g, g.shape[0]

    def compute_flow(self, init=None, gt=None):
        """GNC x coarse-to-fine x IRLS on the GPU (hs.py:49-99, ba.py:57-138,
        classic_nl.py:89-198, alt_ba.py:81-187).  Prints what the reference
        prints (display lines, the per-GNC-stage report with AAE/STD/EPE
        against `gt`) from the library's progress events (of_set_progress)."""
        images, H, W, nc = self._images_planar()
        guide, gc = self._guide_planar(H, W)
        P = self.to_params()
        init_p = None if init is None else nat.planar(init)
        out = np.empty((2, H, W), dtype=np.float32)
        st = _abi.OfStats()
        ctx = nat.context()
        fn, flags = progress_printer(self, gt)
        with ctx.progress(fn, flags):
            ctx.check(ctx.lib.of_compute_flow(ctx.handle, C.byref(P), nat.ptr(images), H, W, nc,
                                              nat.ptr(guide), gc, nat.ptr(init_p), nat.ptr(out), C.byref(st)))
        self.alpha = P.alpha
        if self._METHOD in ('hs', 'alt_ba') or getattr(self, 'auto_level', False):
            self.pyramid_levels = P.pyramid_levels
        self.last_stats = st.as_dict()
        return nat.interleaved(out)

    def compute_flow_base(self, uv):
        """One pyramid level (hs.py:109-142, ba.py:143-206, classic_nl.py:200-277)
        with the current images / color_images / alpha."""
        images, H, W, nc = self._images_planar()
        guide, gc = self._guide_planar(H, W)
        P = self.to_params()
        uvp = nat.planar(uv)
        out = np.empty((2, H, W), dtype=np.float32)
        ctx = nat.context()
        fn, flags = progress_printer(self, None)
        with ctx.progress(fn, flags):
            ctx.check(ctx.lib.of_compute_flow_base(ctx.handle, C.byref(P), nat.ptr(images), H, W, nc,
                                                   nat.ptr(guide), gc, float(self.alpha), nat.ptr(uvp), nat.ptr(out)))
        return nat.interleaved(out)

    def _operator_planes(self, uv, duv, It, Ix, Iy, alpha):
        uv = np.asarray(uv, dtype=float)
        H, W = uv.shape[:2]
        It = np.asarray(It, dtype=float)
        nc = 1 if It.ndim == 2 else It.shape[2]
        P = self.to_params()
        coef = np.empty((7, H, W), dtype=np.float32)
        rhs = np.empty((2, H, W), dtype=np.float32)
        ctx = nat.context()
        ctx.check(ctx.lib.of_flow_operator(
            ctx.handle, C.byref(P), float(alpha), nat.ptr(nat.planar(uv)),
            nat.ptr(None if duv is None else nat.planar(duv)), nat.ptr(nat.planar(It)),
            nat.ptr(nat.planar(Ix)), nat.ptr(nat.planar(Iy)), H, W, nc, nat.ptr(coef), nat.ptr(rhs)))
        return coef, rhs

    def _operator_dia(self, uv, duv, It, Ix, Iy, alpha):
        uv = np.asarray(uv, dtype=float)
        H, W = uv.shape[:2]
        It = np.asarray(It, dtype=float)
        nc = 1 if It.ndim == 2 else It.shape[2]
        P = self.to_params()
        D = max([max(np.atleast_2d(f).shape) - 1 for f in self.spatial_filters] + [0])
        planes = np.empty((dia_nplanes(D), H, W), dtype=np.float32)
        rhs = np.empty((2, H, W), dtype=np.float32)
        d_out = C.c_int(0)
        ctx = nat.context()
        ctx.check(ctx.lib.of_flow_operator_dia(
            ctx.handle, C.byref(P), float(alpha), nat.ptr(nat.planar(uv)),
            nat.ptr(None if duv is None else nat.planar(duv)), nat.ptr(nat.planar(It)),
            nat.ptr(nat.planar(Ix)), nat.ptr(nat.planar(Iy)), H, W, nc, C.byref(d_out), nat.ptr(planes),
            nat.ptr(rhs)))
        assert d_out.value == D
        return D, planes, rhs

    def flow_operator(self, uv, duv, It, Ix, Iy):
        """Assemble A, b on the GPU (matrix-free planes) and return them in the
        reference's scipy form: A (2N x 2N, Fortran-ordered [u; v]), b, None,
        iterative (classic_nl.py:279-378, ba.py:208-302).  A general
        spatial_filters list comes back from the GPU in DIA form
        (of_flow_operator_dia)."""
        alpha = 0.0 if self._METHOD == 'hs' else self._operator_alpha()
        if self._general_filters():
            D, planes, rhs = self._operator_dia(uv, duv, It, Ix, Iy, alpha)
            A = dia_to_sparse(planes, D)
        else:
            coef, rhs = self._operator_planes(uv, duv, It, Ix, Iy, alpha)
            A = planes_to_sparse(coef)
        b = np.concatenate([rhs[0].ravel(order='F'), rhs[1].ravel(order='F')]).astype(float)
        quad = ('quadratic', 'gaussian')
        iterative = not all(r.method in quad for r in list(self.rho_spatial_u) + list(self.rho_spatial_v) + [self.rho_data])
        return A, b, None, iterative

    def _operator_alpha(self):
        return 0.0  # flow_operator(...) evaluates the robust (alpha = 0) system

    def _solve_linear_system(self, A, b, uv_shape, x0=None):
        """base.py:87-114 on the GPU: A must have the 5-point + 2x2-coupling
        structure that flow_operator produces."""
        H, W = int(uv_shape[0]), int(uv_shape[1])
        bb = np.asarray(b, dtype=float)
        rhs = np.stack([bb[:H * W].reshape(H, W, order='F'), bb[H * W:].reshape(H, W, order='F')])
        P = self.to_params()
        x = np.empty((2, H, W), dtype=np.float32)
        it = C.c_int(0)
        rr = C.c_double(0)
        ctx = nat.context()
        try:
            coef = sparse_to_planes(A, H, W)
        except NotImplementedError:
            # any other 2-D stencil operator (general spatial_filters): DIA form
            D, planes = sparse_to_dia(A, H, W)
            ctx.check(ctx.lib.of_solve_dia(ctx.handle, C.byref(P), D, nat.ptr(nat.f32(planes)),
                                           nat.ptr(nat.f32(rhs)), H, W, nat.ptr(x), C.byref(it), C.byref(rr)))
        else:
            ctx.check(ctx.lib.of_solve(ctx.handle, C.byref(P), nat.ptr(nat.f32(coef)), nat.ptr(nat.f32(rhs)), H, W,
                                       nat.ptr(x), C.byref(it), C.byref(rr)))
        # iterations (CG) / sweeps (SOR) and the solver's own residual estimate
        self.last_solve = {"iters": it.value, "rel_residual": rr.value}
        return nat.interleaved(x).reshape(uv_shape)


def planes_to_sparse(coef):
    """7 coefficient planes -> scipy CSC matrix with the reference's ordering
    (column-major pixel index k = j*H + i, u block then v block)."""
    coef = np.asarray(coef, dtype=float)
    _, H, W = coef.shape
    N = H * W
    k = np.arange(N).reshape(W, H).T  # k[i, j] = j*H + i
    rows, cols, vals = [], [], []

    def add(r, c, v):
        rows.append(r.ravel())
        cols.append(c.ravel())
        vals.append(v.ravel())

    for comp, (wx, wy) in enumerate(((coef[0], coef[1]), (coef[2], coef[3]))):
        o = comp * N
        kr, kc = k[:, :-1], k[:, 1:]
        add(o + kr, o + kc, -wx[:, :-1]); add(o + kc, o + kr, -wx[:, :-1])
        kr, kc = k[:-1, :], k[1:, :]
        add(o + kr, o + kc, -wy[:-1, :]); add(o + kc, o + kr, -wy[:-1, :])
    add(k, k, coef[4]); add(N + k, N + k, coef[6])
    add(k, N + k, coef[5]); add(N + k, k, coef[5])
    return sparse.csc_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(2 * N, 2 * N))


def sparse_to_planes(A, H, W):
    """Inverse of planes_to_sparse; raises NotImplementedError when A is not a
    symmetric 5-point + 2x2-coupling operator."""
    N = H * W
    A = sparse.csr_matrix(A)
    if A.shape != (2 * N, 2 * N):
        raise ValueError(f"A has shape {A.shape}, expected {(2 * N, 2 * N)}")
    k = np.arange(N).reshape(W, H).T
    d = A.diagonal()
    coef = np.zeros((7, H, W))
    coef[4] = d[:N].reshape(H, W, order='F')
    coef[6] = d[N:].reshape(H, W, order='F')
    coef[5] = np.asarray(A[k.ravel(), N + k.ravel()]).reshape(H, W)
    for comp in range(2):
        o = comp * N
        coef[2 * comp][:, :-1] = -np.asarray(A[o + k[:, :-1].ravel(), o + k[:, 1:].ravel()]).reshape(H, W - 1)
        coef[2 * comp + 1][:-1, :] = -np.asarray(A[o + k[:-1, :].ravel(), o + k[1:, :].ravel()]).reshape(H - 1, W)
    R = planes_to_sparse(coef)
    if abs(R - A).max() > 1e-9 * max(1.0, abs(A).max()):
        raise NotImplementedError("A is not a symmetric 5-point + 2x2-coupling flow operator")
    return coef


def dia_nplanes(D):
    """planes of the DIA operator of radius D: G u-u, G v-v, 1 u-v (G = (2D+1)^2)"""
    return 2 * (2 * D + 1) ** 2 + 1


def dia_to_sparse(planes, D):
    """DIA planes (include/optflow.h, of_flow_operator_dia) -> scipy CSC with
    the reference's ordering (k = j*H + i, u block then v block)."""
    planes = np.asarray(planes, dtype=float)
    _, H, W = planes.shape
    N = H * W
    S = 2 * D + 1
    G = S * S
    k = np.arange(N).reshape(W, H).T
    rows, cols, vals = [], [], []
    for comp in range(2):
        o = comp * N
        for di in range(-D, D + 1):
            for dj in range(-D, D + 1):
                c = planes[comp * G + (di + D) * S + (dj + D)]
                i0, i1 = max(0, -di), min(H, H - di)
                j0, j1 = max(0, -dj), min(W, W - dj)
                if i0 >= i1 or j0 >= j1:
                    continue
                blk = c[i0:i1, j0:j1]
                nz = blk != 0
                rows.append(o + k[i0:i1, j0:j1][nz])
                cols.append(o + k[i0 + di:i1 + di, j0 + dj:j1 + dj][nz])
                vals.append(blk[nz])
    cuv = planes[2 * G]
    nz = cuv != 0
    rows += [k[nz], N + k[nz]]
    cols += [N + k[nz], k[nz]]
    vals += [cuv[nz], cuv[nz]]
    return sparse.csc_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                             shape=(2 * N, 2 * N))


def sparse_to_dia(A, H, W):
    """Inverse of dia_to_sparse for any A whose u-u and v-v blocks are 2-D
    stencils of radius <= 4 and whose u-v block is diagonal; raises
    NotImplementedError otherwise.  Returns (D, planes)."""
    N = H * W
    A = sparse.coo_matrix(A)
    if A.shape != (2 * N, 2 * N):
        raise ValueError(f"A has shape {A.shape}, expected {(2 * N, 2 * N)}")
    r, c, v = A.row, A.col, A.data
    rc, cc = r // N, c // N
    ri, rj = (r % N) % H, (r % N) // H
    ci, cj = (c % N) % H, (c % N) // H
    di, dj = ci - ri, cj - rj
    same = rc == cc
    if np.any(~same & ((di != 0) | (dj != 0))):
        raise NotImplementedError("A's u-v block is not diagonal")
    D = int(max(np.abs(di).max(initial=0), np.abs(dj).max(initial=0)))
    if D > 4:
        raise NotImplementedError("A couples pixels more than 4 apart")
    S = 2 * D + 1
    G = S * S
    planes = np.zeros((dia_nplanes(D), H, W))
    e = np.where(same, rc * G + (di + D) * S + (dj + D), 2 * G)
    keep = same | (rc == 0)  # the u-v coupling once, from the u rows
    np.add.at(planes, (e[keep], ri[keep], rj[keep]), v[keep])
    R = dia_to_sparse(planes, D)
    if abs(R - A).max() > 1e-9 * max(1.0, abs(A).max()):
        raise NotImplementedError("A is not a 2-D stencil operator of the flow system's form")
    return D, planes
