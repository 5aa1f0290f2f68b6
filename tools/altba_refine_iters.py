"""Offline experiment: AltBA alpha = 0 (condition ~3.6e6)
with the 'backslash' surrogate.  float32 PCG (degree-5 Chebyshev block-Jacobi
preconditioner, as k_cg_small) with the residual replaced by the fp64 true
residual b - A (x_hi + x_lo) every time the recursive one has fallen by
`upd_rel` (x_hi accumulated in fp64), vs spsolve on the float64 system
(the reference) and on the float32-rounded system (the float32 floor).

The system: the first warp of AltBAOpticalFlow.compute_flow_base on the
tests/golden/altba.npz level (alt_ba.py:214-243), assembled by the reference
itself (imported from /root/reference: build container only).
usage: PYTHONDONTWRITEBYTECODE=1 python tools/altba_refine_iters.py"""
import os
import sys

import numpy as np
from scipy import sparse
from scipy.sparse.linalg import spsolve

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, "/root/reference")
import optical_flow as ref  # noqa: E402  (the reference)
from optical_flow.methods import config as ref_cfg  # noqa: E402
from optical_flow.utils.derivatives import partial_deriv  # noqa: E402
from optical_flow.robust.robust_function import RobustFunction  # noqa: E402

assert ref.__file__.startswith("/root/reference")


def cheb(m, a, b=2.0):
    """tools/poly_iters.py's Chebyshev preconditioner coefficients in B"""
    from numpy.polynomial import chebyshev as Ch
    from numpy.polynomial import polynomial as Pl
    s = (b + a) / (b - a)
    gg = -2.0 / (b - a)
    T = np.zeros(m + 2)
    T[m + 1] = 1
    P = Ch.cheb2poly(T)
    Ts = np.polyval(P[::-1], s)
    R = np.zeros(1)
    for k, c in enumerate(P):
        R = Pl.polyadd(R, c * Pl.polypow([s, gg], k))
    R = R / Ts
    pX = -R[1:]
    cB = np.zeros(m + 1)
    for j, c in enumerate(pX):
        cB[:len(Pl.polypow([1, -1], j))] += c * Pl.polypow([1, -1], j)
    return cB


def block_parts(A, n):
    a_, c_, d_ = A.diagonal()[:n], A[:n, n:].diagonal(), A.diagonal()[n:]
    det = a_ * d_ - c_ * c_
    Dinv = sparse.bmat([[sparse.diags(d_ / det), sparse.diags(-c_ / det)],
                        [sparse.diags(-c_ / det), sparse.diags(a_ / det)]]).tocsr()
    D = sparse.bmat([[sparse.diags(a_), sparse.diags(c_)], [sparse.diags(c_), sparse.diags(d_)]]).tocsr()
    return D, Dinv


def system(alpha):
    d = np.load(os.path.join(ROOT, "tests", "golden", "altba.npz"))
    o = ref_cfg.load_of_method("classic-c-a")
    o.images = d["base_images"]
    o.lambda2 = 0.01
    o.max_iters = 4
    o.alpha = alpha
    uv, uvhat = d["base_uv"].copy(), d["base_uvhat"].copy()
    lambda2 = 1e-4  # Lambda2s[0]
    It, Ix, Iy = partial_deriv(o.images, uv, o.interpolation_method, o.deriv_filter)
    duv = np.zeros_like(uv)
    qua = __import__("copy").copy(o)
    qua.lambda_ = o.lambda_q
    qua.rho_spatial_u = [RobustFunction('quadratic', 1) for _ in o.rho_spatial_u]
    qua.rho_spatial_v = [RobustFunction('quadratic', 1) for _ in o.rho_spatial_v]
    qua.rho_data = RobustFunction('quadratic', 1)
    if alpha == 1:
        A, b, _, _ = qua.flow_operator(uv, duv, It, Ix, Iy)
    else:
        A, b, _, _ = o.flow_operator(uv, duv, It, Ix, Iy)
    tmp = o.rho_couple.deriv_over_x(uv.ravel(order='F') - uvhat.ravel(order='F'))
    A = (A + lambda2 * sparse.diags(tmp, 0, shape=A.shape)).tocsr()
    b = b + lambda2 * tmp * (uvhat.ravel(order='F') - uv.ravel(order='F'))
    return A, b, uv.shape[:2]


def pcg32(A64, b, upd_rel, rtol, maxit=20000, deg=5, lo=0.02):
    A = A64.astype(np.float32).tocsr()
    n = A.shape[0] // 2
    D, Dinv = block_parts(A.astype(np.float64), n)
    Dinv = Dinv.astype(np.float32)
    B = (Dinv @ (D.astype(np.float32) - A)).tocsr().astype(np.float32)
    cB = cheb(deg, lo).astype(np.float32)

    def M(r):
        y = Dinv @ r
        g = cB[deg] * y
        for i in range(deg - 1, -1, -1):
            g = cB[i] * y + B @ g
        return g.astype(np.float32)
    A64r = A.astype(np.float64)  # the fp32 operator, evaluated in fp64
    bn = np.linalg.norm(b)
    xh = np.zeros(2 * n)           # x_hi, fp64
    x = np.zeros(2 * n, np.float32)  # x_lo
    r = b.astype(np.float32)
    z = M(r)
    p = z.copy()
    rz = np.float32(r @ z)
    r_ref = bn
    nupd = 0
    for k in range(maxit):
        rr = float(np.linalg.norm(r.astype(np.float64)))
        if upd_rel > 0 and rr < upd_rel * r_ref:
            xh = xh + x.astype(np.float64)
            x[:] = 0
            rt = b - A64r @ xh
            r = rt.astype(np.float32)
            rr = np.linalg.norm(rt)
            r_ref = rr
            nupd += 1
        true = np.linalg.norm(b - A64r @ (xh + x.astype(np.float64))) / bn
        if rr < rtol * bn:
            return xh + x, k, true, nupd
        q = (A @ p).astype(np.float32)
        al = np.float32(rz / np.float32(p @ q))
        x = (x + al * p).astype(np.float32)
        r = (r - al * q).astype(np.float32)
        z = M(r)
        rz2 = np.float32(r @ z)
        p = (z + np.float32(rz2 / rz) * p).astype(np.float32)
        rz = rz2
    return xh + x, maxit, np.linalg.norm(b - A64r @ (xh + x)) / bn, nupd


def main():
    for alpha in (0.0, 1.0):
        A, b, (H, W) = system(alpha)
        x64 = spsolve(A.tocsc(), b)
        x32 = spsolve(A.astype(np.float32).astype(np.float64).tocsc(), b)

        def epe(x):
            d = (x - x64).reshape(2, -1)
            return float(np.sqrt((d ** 2).sum(0)).mean())
        print(f"alpha {alpha}: float32-operator floor {epe(x32):.3e} px mean", flush=True)
        for rtol, upd in ((1e-6, 1e-3), (1e-6, 0.0), (1e-8, 1e-3), (1e-10, 1e-3), (1e-12, 1e-3)):
            x, k, true, nu = pcg32(A, b, upd, rtol)
            print(f"  rtol {rtol:g} upd_rel {upd:g}: iters {k} replacements {nu} true rel residual {true:.2e} "
                  f"EPE to spsolve {epe(x):.3e}", flush=True)


if __name__ == "__main__":
    main()
