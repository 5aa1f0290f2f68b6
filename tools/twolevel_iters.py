"""Offline prototype: does a coarse-grid correction cut
the robust-stage CG iterations of the 'backslash' surrogate enough to pay
for a second pass over the fine level?

Operator: Classic+NL-fast at 540x960 assembled by the float64 oracle (as
tools/poly_iters.py: synthetic pair, texture images, perturbed GT flow), GNC
stages alpha = 1 (quadratic) and 0 (robust).  Preconditioners, CG to 1e-6:
  poly5      the production one: degree-5 Chebyshev in B = D^-1 N (k_cgs)
  2lv-s<d>   symmetric two-level: degree-d polynomial pre-smoothing, coarse
             correction on 2x2-pixel aggregates (Galerkin P^T A P, piecewise
             constant P, coarse system solved exactly), post-smoothing
  vc-s<d>    the same with the coarse system itself handled by a V-cycle
             down to <= 2000 unknowns (recursively aggregated)
Per iteration a two-level step costs ~2 fine passes (pre-smooth+residual+
restrict, prolong+post-smooth+CG update) vs one for poly5.
usage: python tools/twolevel_iters.py [H W]"""
import os
import sys
import time

import numpy as np
from scipy import sparse
from scipy.sparse.linalg import splu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'optical-flow-python_amd'), os.path.join(ROOT, 'oracle')]
import oracle as O  # noqa: E402
from optical_flow.methods.config import load_of_method  # noqa: E402
from optical_flow.methods.base import planes_to_sparse  # noqa: E402
from optical_flow.utils.synthetic import synth_pair  # noqa: E402

H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (540, 960)


def cheb(m, a, b=2.0):
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
    """D (2x2 blocks), D^-1 of A = [[Auu, Auv], [Avu, Avv]] (u block then v)."""
    a_, c_, d_ = A.diagonal()[:n], A[:n, n:].diagonal(), A.diagonal()[n:]
    det = a_ * d_ - c_ * c_
    Dinv = sparse.bmat([[sparse.diags(d_ / det), sparse.diags(-c_ / det)],
                        [sparse.diags(-c_ / det), sparse.diags(a_ / det)]]).tocsr()
    D = sparse.bmat([[sparse.diags(a_), sparse.diags(c_)], [sparse.diags(c_), sparse.diags(d_)]]).tocsr()
    return D, Dinv


def agg_P(h, w):
    """Piecewise-constant prolongation, 2x2 aggregates, Fortran-order pixels
    (the reference's ravel(order='F')), both components."""
    hc, wc = (h + 1) // 2, (w + 1) // 2
    ii, jj = np.meshgrid(np.arange(h), np.arange(w), indexing='ij')
    fine = (ii + jj * h).ravel()
    coarse = (ii // 2 + (jj // 2) * hc).ravel()
    Ps = sparse.csr_matrix((np.ones(h * w), (fine, coarse)), shape=(h * w, hc * wc))
    return sparse.block_diag([Ps, Ps]).tocsr(), hc, wc


class Level:
    def __init__(self, A, h, w, deg, lo):
        self.A, self.h, self.w = A, h, w
        n = h * w
        self.D, self.Dinv = block_parts(A, n)
        self.B = (self.Dinv @ (self.D - A)).tocsr()
        self.cB = cheb(deg, lo)
        self.deg = deg

    def smooth(self, r):
        """poly(B) D^-1 r (SPD)"""
        y = self.Dinv @ r
        g = self.cB[self.deg] * y
        for i in range(self.deg - 1, -1, -1):
            g = self.cB[i] * y + self.B @ g
        return g


def build_hierarchy(A, h, w, deg, lo, exact_levels, min_n=2000):
    levels = [Level(A, h, w, deg, lo)]
    Ps = []
    while True:
        L = levels[-1]
        if 2 * L.h * L.w <= min_n or len(levels) > exact_levels:
            break
        P, hc, wc = agg_P(L.h, L.w)
        Ac = (P.T @ L.A @ P).tocsr()
        Ps.append(P)
        levels.append(Level(Ac, hc, wc, deg, lo))
    return levels, Ps, splu(levels[-1].A.tocsc())


def vcycle(levels, Ps, lu, lev, r, omega_c):
    if lev == len(levels) - 1:
        return lu.solve(r)
    L = levels[lev]
    x = L.smooth(r)
    rc = Ps[lev].T @ (r - L.A @ x)
    x = x + omega_c * (Ps[lev] @ vcycle(levels, Ps, lu, lev + 1, rc, omega_c))
    return x + L.smooth(r - L.A @ x)


def pcg(A, b, Minv, maxit=3000, rtol=1e-6):
    x = np.zeros_like(b)
    r = b.copy()
    z = Minv(r)
    p = z.copy()
    rz = r @ z
    bn = np.linalg.norm(b)
    for k in range(maxit):
        if np.linalg.norm(r) < rtol * bn:
            return k
        q = A @ p
        al = rz / (p @ q)
        x += al * p
        r -= al * q
        z = Minv(r)
        rz2 = r @ z
        p = z + (rz2 / rz) * p
        rz = rz2
    return maxit


def main():
    im1, im2, gt = synth_pair(H, W, 0)
    g = lambda im: np.floor(0.2989 * im[..., 0] + 0.5870 * im[..., 1] + 0.1140 * im[..., 2] + 0.5)  # noqa: E731
    imgs = np.stack([g(im1), g(im2)], 2)
    tex = O.rof_texture(imgs)
    o = load_of_method('classic+nl-fast')
    uv = gt + 0.3 * np.sin(np.arange(H)[:, None, None] / 17.0)
    It, Ix, Iy = O.partial_deriv(tex, uv, 'bi-cubic')
    for alpha in (1.0, 0.0):
        coef, rhs = O.flow_operator(o.to_params(), alpha, uv, None, It, Ix, Iy)
        A = planes_to_sparse(coef).tocsr()
        b = np.concatenate([rhs[0].ravel(order='F'), rhs[1].ravel(order='F')])
        lo = 0.04 if alpha >= 0.5 else 0.02
        L0 = Level(A, H, W, 5, lo)
        t = time.time()
        print(f"alpha {alpha}: poly5 iters {pcg(A, b, L0.smooth)} ({time.time() - t:.1f}s)", flush=True)
        for deg in (1, 2, 3):
            for exact_levels, tag in ((1, '2lv'), (99, 'vc')):
                levels, Ps, lu = build_hierarchy(A, H, W, deg, lo, exact_levels)
                for om in (1.0, 1.5, 2.0):
                    t = time.time()
                    k = pcg(A, b, lambda r: vcycle(levels, Ps, lu, 0, r, om))
                    print(f"alpha {alpha}: {tag}-s{deg} levels {len(levels)} omega_c {om}: iters {k} "
                          f"({time.time() - t:.1f}s)", flush=True)


if __name__ == "__main__":
    main()
