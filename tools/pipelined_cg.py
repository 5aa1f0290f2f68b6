"""Pipelined CG for the 'backslash' surrogate, prototyped before building
(VERDICT r5 "next" 3): iterations and attainable true residual of
Ghysels-Vanroose pipelined PCG (one global reduction per iteration,
overlapped with the operator + preconditioner of the same iteration) against
standard PCG, both with k_cgs's preconditioner (2x2 block Jacobi + degree-5
Chebyshev polynomial on [0.01, 2], robust stage; [0.04, 2] quadratic), on
the Classic+NL-fast operator the float64 oracle assembles at 540x960
(synthetic pair, texture images, perturbed GT flow -- tools/poly_iters.py's
setup).  Vectors in float64 and rounded to float32 after every update (the
GPU stores r, x, p and the extra pipelined vectors in fp32).

Why it matters: k_cgs already overlaps iteration k's reductions with
iteration k+1's launch (lag 1: the partial sums of launch k are finished in
launch k+1's prologue); a band could start iteration k+1 before every band
of iteration k has finished only with lag-2 scalars, i.e. p(2)-CG, whose
extra recurrences cost bytes per pixel and accuracy.  This measures the
lag-1 pipelined form's attainable accuracy as the optimistic bound.
usage: python tools/pipelined_cg.py [--size 540x960]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'optical-flow-python_amd'), os.path.join(ROOT, 'oracle')]
import numpy as np  # noqa: E402
from scipy import sparse  # noqa: E402

import oracle as O  # noqa: E402
from optical_flow.methods.base import planes_to_sparse  # noqa: E402
from optical_flow.methods.config import load_of_method  # noqa: E402
from optical_flow.utils.synthetic import synth_pair  # noqa: E402


def cheb(m, a, b=2.0):
    """p(B) coefficients of the degree-m Chebyshev residual polynomial on
    [a, b] (driver.hip cheb_poly)."""
    from numpy.polynomial import chebyshev as Ch
    from numpy.polynomial import polynomial as Pl
    s, gg = (b + a) / (b - a), -2.0 / (b - a)
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="540x960")
    ap.add_argument("--rtol", type=float, default=1e-6)
    a = ap.parse_args()
    H, W = map(int, a.size.split("x"))
    im1, im2, gt = synth_pair(H, W, 0)
    g = lambda im: np.floor(0.2989 * im[..., 0] + 0.5870 * im[..., 1] + 0.1140 * im[..., 2] + 0.5)  # noqa: E731
    tex = O.rof_texture(np.stack([g(im1), g(im2)], 2))
    o = load_of_method('classic+nl-fast')
    uv = gt + 0.3 * np.sin(np.arange(H)[:, None, None] / 17.0)
    It, Ix, Iy = O.partial_deriv(tex, uv, 'bi-cubic')
    for alpha, lo in ((1.0, 0.04), (0.0, 0.01)):
        coef, rhs = O.flow_operator(o.to_params(), alpha, uv, None, It, Ix, Iy)
        A = planes_to_sparse(coef).tocsr()
        b = np.concatenate([rhs[0].ravel(order='F'), rhs[1].ravel(order='F')])
        a_, c_, d_ = coef[4].ravel(order='F'), coef[5].ravel(order='F'), coef[6].ravel(order='F')
        det = a_ * d_ - c_ * c_
        Dinv = sparse.bmat([[sparse.diags(d_ / det), sparse.diags(-c_ / det)],
                            [sparse.diags(-c_ / det), sparse.diags(a_ / det)]]).tocsr()
        D = sparse.bmat([[sparse.diags(a_), sparse.diags(c_)], [sparse.diags(c_), sparse.diags(d_)]]).tocsr()
        B = (Dinv @ (D - A)).tocsr()
        m = 5
        cB = cheb(m, lo)

        def Minv(r):
            y = Dinv @ r
            gg = cB[m] * y
            for i in range(m - 1, -1, -1):
                gg = cB[i] * y + B @ gg
            return gg
        bn = np.linalg.norm(b)

        def rnd(v, f32):
            return v.astype(np.float32).astype(np.float64) if f32 else v

        def pcg(f32):
            x = np.zeros_like(b)
            r = b.copy()
            z = Minv(r)
            p = z.copy()
            rz = r @ z
            for k in range(3000):
                if np.linalg.norm(r) < a.rtol * bn:
                    break
                q = A @ p
                al = rz / (p @ q)
                x = rnd(x + al * p, f32)
                r = rnd(r - al * q, f32)
                z = Minv(r)
                rz2 = r @ z
                p = rnd(z + (rz2 / rz) * p, f32)
                rz = rz2
            return k, np.linalg.norm(b - A @ x) / bn, np.linalg.norm(r) / bn

        def pipecg(f32, maxit=3000):
            """Ghysels & Vanroose (2014) Alg. 4, preconditioned: u = M r,
            w = A u; the dots gamma = r.u, delta = w.u of one iteration
            overlap m = M w, n = A m."""
            x = np.zeros_like(b)
            r = b.copy()
            u = Minv(r)
            w = A @ u
            z = q = s = p = np.zeros_like(b)
            gam_old = al = 1.0
            for k in range(maxit):
                gam, delta = r @ u, w @ u
                if np.sqrt(abs(r @ r)) < a.rtol * bn:
                    break
                mm = Minv(w)
                nn = A @ mm
                if k > 0:
                    be = gam / gam_old
                    al = gam / (delta - be * gam / al)
                else:
                    be = 0.0
                    al = gam / delta
                z = rnd(nn + be * z, f32)
                q = rnd(mm + be * q, f32)
                s = rnd(w + be * s, f32)
                p = rnd(u + be * p, f32)
                x = rnd(x + al * p, f32)
                r = rnd(r - al * s, f32)
                u = rnd(u - al * q, f32)
                w = rnd(w - al * z, f32)
                gam_old = gam
            return k, np.linalg.norm(b - A @ x) / bn, np.linalg.norm(r) / bn
        for f32 in (False, True):
            t = time.time()
            k, tr, er = pcg(f32)
            print(f"alpha {alpha} {'fp32' if f32 else 'fp64'} PCG          iters {k:4d}  true rel {tr:.2e}  "
                  f"recursive {er:.2e}  ({time.time() - t:.0f} s)", flush=True)
            t = time.time()
            k, tr, er = pipecg(f32)
            print(f"alpha {alpha} {'fp32' if f32 else 'fp64'} pipelined PCG iters {k:4d}  true rel {tr:.2e}  "
                  f"recursive {er:.2e}  ({time.time() - t:.0f} s)", flush=True)


if __name__ == "__main__":
    main()
