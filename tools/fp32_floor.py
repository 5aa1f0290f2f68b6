"""How close to the true solution can an fp32 iterate get?  On the Classic+NL
operator of tools/poly_iters.py (540x960, oracle-assembled, fp64) for the
quadratic (alpha 1) and robust (alpha 0) GNC stages:
  - floor: ||b - A fl32(x*)|| / ||b|| with x* the fp64 solution (CG to 1e-13);
  - fp32 CG (the degree-5 preconditioner, x, r, p in fp32): the recursive
    residual vs the fp64 true residual of x at each 1e-6 crossing, with and
    without residual replacement r <- b - A x (fp64-evaluated, stored fp32).
CPU only.  usage: python tools/fp32_floor.py [H W]"""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'optical-flow-python_amd'), os.path.join(ROOT, 'oracle')]
import numpy as np, oracle as O
from scipy import sparse
from optical_flow.methods.config import load_of_method
from optical_flow.methods.base import planes_to_sparse
from optical_flow.utils.synthetic import synth_pair

H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (540, 960)
im1, im2, gt = synth_pair(H, W, 0)
g = lambda im: np.floor(0.2989 * im[..., 0] + 0.5870 * im[..., 1] + 0.1140 * im[..., 2] + 0.5)
imgs = np.stack([g(im1), g(im2)], 2)
tex = O.rof_texture(imgs)
o = load_of_method('classic+nl-fast')
uv = gt + 0.3 * np.sin(np.arange(H)[:, None, None] / 17.0)
It, Ix, Iy = O.partial_deriv(tex, uv, 'bi-cubic')


def cheb(m, a, b=2.0):
    from numpy.polynomial import chebyshev as Ch, polynomial as Pl
    s = (b + a) / (b - a); gg = -2.0 / (b - a)
    T = np.zeros(m + 2); T[m + 1] = 1
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


for alpha in (1.0, 0.0):
    coef, rhs = O.flow_operator(o.to_params(), alpha, uv, None, It, Ix, Iy)
    A = planes_to_sparse(coef).tocsr()
    b = np.concatenate([rhs[0].ravel(order='F'), rhs[1].ravel(order='F')])
    a_, c_, d_ = coef[4].ravel(order='F'), coef[5].ravel(order='F'), coef[6].ravel(order='F')
    det = a_ * d_ - c_ * c_
    Dinv = sparse.bmat([[sparse.diags(d_ / det), sparse.diags(-c_ / det)], [sparse.diags(-c_ / det), sparse.diags(a_ / det)]]).tocsr()
    D = sparse.bmat([[sparse.diags(a_), sparse.diags(c_)], [sparse.diags(c_), sparse.diags(d_)]]).tocsr()
    B = (Dinv @ (D - A)).tocsr()
    m = 5
    cB = cheb(m, 0.04)
    A32, Dinv32, B32 = A.astype(np.float32), Dinv.astype(np.float32), B.astype(np.float32)
    bn = np.linalg.norm(b)

    def Minv(r, Di, Bm, dt):
        y = Di @ r
        gg = dt(cB[m]) * y
        for i in range(m - 1, -1, -1):
            gg = dt(cB[i]) * y + Bm @ gg
        return gg

    # fp64 solution
    x = np.zeros_like(b); r = b.copy(); z = Minv(r, Dinv, B, np.float64); p = z.copy(); rz = r @ z
    for k in range(3000):
        if np.linalg.norm(r) < 1e-13 * bn: break
        q = A @ p; al = rz / (p @ q); x += al * p; r -= al * q; z = Minv(r, Dinv, B, np.float64); rz2 = r @ z; p = z + (rz2 / rz) * p; rz = rz2
    xs = x.copy()
    true = lambda xx: np.linalg.norm(b - A @ xx.astype(np.float64)) / bn
    print(f'alpha {alpha}: fp64 CG {k} its, true {true(xs):.2e}; fl32(x*) floor {true(xs.astype(np.float32)):.2e}; '
          f'|A||x|/|b| ~ {np.linalg.norm(abs(A) @ abs(xs)) / bn:.1f}', flush=True)
    b32 = b.astype(np.float32)
    for every in (0, 10, 25):
        x = np.zeros_like(b32); r = b32.copy(); z = Minv(r, Dinv32, B32, np.float32); p = z.copy(); rz = float(r.astype(np.float64) @ z)
        log = []
        for k in range(400):
            rn = np.linalg.norm(r.astype(np.float64))
            if rn < 1e-6 * bn:
                log.append((k, rn / bn, true(x)))
                break
            if every and k and k % every == 0:
                r = (b - A @ x.astype(np.float64)).astype(np.float32)
            q = A32 @ p; al = np.float32(rz / float(p.astype(np.float64) @ q)); x = x + al * p; r = r - al * q
            z = Minv(r, Dinv32, B32, np.float32); rz2 = float(r.astype(np.float64) @ z); p = z + np.float32(rz2 / rz) * p; rz = rz2
        print(f'  fp32 CG replace every {every}: stop at {log}', flush=True)
    # reliable updates: fp32 CG on (x_lo, r, p); when ||r|| falls below delta x
    # the largest ||r|| since the last update, x_hi += x_lo (fp64), r = b - A
    # x_hi (fp64-evaluated, stored fp32), x_lo = 0; p and the recurrence kept
    for delta in (0.1, 0.03, 0.01):
        xh = np.zeros_like(b); xl = np.zeros_like(b32); r = b32.copy(); z = Minv(r, Dinv32, B32, np.float32); p = z.copy()
        rz = float(r.astype(np.float64) @ z); rmax = np.linalg.norm(b); nup = 0
        for k in range(400):
            rn = np.linalg.norm(r.astype(np.float64))
            rmax = max(rmax, rn)
            if rn < delta * rmax or rn < 1e-6 * bn:
                xh += xl; xl[:] = 0; nup += 1
                r = (b - A @ xh).astype(np.float32); rn = np.linalg.norm(r.astype(np.float64)); rmax = rn
                if rn < 1e-6 * bn:
                    break
            q = A32 @ p; al = np.float32(rz / float(p.astype(np.float64) @ q)); xl = xl + al * p; r = r - al * q
            z = Minv(r, Dinv32, B32, np.float32); rz2 = float(r.astype(np.float64) @ z); p = z + np.float32(rz2 / rz) * p; rz = rz2
        print(f'  reliable updates delta {delta}: {k} its, {nup} updates, true(x_hi) {true(xh):.2e}, '
              f'true(fl32(x_hi)) {true(xh.astype(np.float32)):.2e}, |x_hi - x*|/|x*| {np.linalg.norm(xh - xs) / np.linalg.norm(xs):.2e}, '
              f'fp32 CG x err {np.linalg.norm(x.astype(np.float64) - xs) / np.linalg.norm(xs):.2e}', flush=True)
