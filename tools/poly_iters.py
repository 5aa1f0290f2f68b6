"""CG iterations to 1e-6 relative residual with the Chebyshev polynomial
preconditioner p(B) D^-1 (2x2 block-Jacobi splitting A = D - N, B = D^-1 N)
of degree 1..7 on a Classic+NL-fast operator assembled by the float64 oracle
at 540x960 (synthetic pair, texture images, perturbed ground-truth flow),
for the quadratic (alpha 1) and robust (alpha 0) GNC stages.  CPU only.
usage: python tools/poly_iters.py"""
import sys, time; import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'optical-flow-python_amd'), os.path.join(ROOT, 'oracle')]
import numpy as np, oracle as O
from scipy import sparse
from optical_flow.methods.config import load_of_method
from optical_flow.methods.base import planes_to_sparse
from optical_flow.utils.synthetic import synth_pair
H,W = 540, 960
im1, im2, gt = synth_pair(H, W, 0)
g = lambda im: np.floor(0.2989*im[...,0]+0.5870*im[...,1]+0.1140*im[...,2]+0.5)
imgs = np.stack([g(im1), g(im2)], 2)
t=time.time(); tex = O.rof_texture(imgs); print('rof', time.time()-t, flush=True)
o = load_of_method('classic+nl-fast')
# start from a perturbed GT so the increment is nontrivial
uv = gt + 0.3*np.sin(np.arange(H)[:,None,None]/17.0)
It, Ix, Iy = O.partial_deriv(tex, uv, 'bi-cubic')
def cheb(m, a, b=2.0):
    from numpy.polynomial import chebyshev as Ch
    # R(X) = T_{m+1}((b+a-2X)/(b-a)) / T_{m+1}((b+a)/(b-a)); p(X) = (1-R(X))/X in powers of X
    s=(b+a)/(b-a); gg=-2.0/(b-a)
    T=np.zeros(m+2); T[m+1]=1
    P=Ch.cheb2poly(T)  # coefficients in t
    Ts=np.polyval(P[::-1], s)
    # substitute t = s + g X
    from numpy.polynomial import polynomial as Pl
    R=np.zeros(1)
    for k,c in enumerate(P):
        R=Pl.polyadd(R, c*Pl.polypow([s,gg],k))
    R=R/Ts
    pX=-R[1:]  # (1-R)/X
    # convert p(X) with X = 1 - B into powers of B
    cB=np.zeros(m+1)
    for j,c in enumerate(pX):
        cB[:len(Pl.polypow([1,-1],j))]+=c*Pl.polypow([1,-1],j)
    return cB
for alpha in (1.0, 0.0):
    coef, rhs = O.flow_operator(o.to_params(), alpha, uv, None, It, Ix, Iy)
    A = planes_to_sparse(coef).tocsr()
    b = np.concatenate([rhs[0].ravel(order='F'), rhs[1].ravel(order='F')])
    n = H*W
    a_, c_, d_ = coef[4].ravel(order='F'), coef[5].ravel(order='F'), coef[6].ravel(order='F')
    det = a_*d_ - c_*c_
    Dinv = sparse.bmat([[sparse.diags(d_/det), sparse.diags(-c_/det)],[sparse.diags(-c_/det), sparse.diags(a_/det)]]).tocsr()
    D = sparse.bmat([[sparse.diags(a_), sparse.diags(c_)],[sparse.diags(c_), sparse.diags(d_)]]).tocsr()
    N = (D - A).tocsr()
    B = (Dinv @ N).tocsr()
    def pcg(m, lo):
        cB = cheb(m, lo)
        def Minv(r):
            y = Dinv @ r
            g = cB[m]*y
            for i in range(m-1, -1, -1):
                g = cB[i]*y + B @ g
            return g
        x=np.zeros_like(b); r=b.copy(); z=Minv(r); p=z.copy(); rz=r@z; bn=np.linalg.norm(b)
        for k in range(3000):
            if np.linalg.norm(r) < 1e-6*bn: return k
            q=A@p; al=rz/(p@q); x+=al*p; r-=al*q; z=Minv(r); rz2=r@z; p=z+(rz2/rz)*p; rz=rz2
        return 3000
    for m in (1,3,5,7):
        for lo in (0.02,0.04,0.08):
            k=pcg(m,lo); print(f'alpha {alpha} degree {m} lo {lo}: iters {k}  stencil-apps/iter {m+1}', flush=True)
