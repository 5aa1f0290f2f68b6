"""(The flow perturbation below varies by row only, which biases the robust
weights towards horizontal coupling; see CGS_PAIR in kernels_solve.hip for the
GPU measurement.)  CG iterations to 1e-6 relative residual with the degree-5 Chebyshev
polynomial preconditioner in the 2x2 block-Jacobi splitting (k_cgs before
CGS_PAIR) vs the pair-block splitting (4x4 blocks of the horizontal pixel
pairs (2k, 2k+1), the edge inside a pair moved into the block) on a
Classic+NL-fast operator assembled by the float64 oracle (synthetic pair,
texture images, perturbed ground-truth flow), quadratic (alpha 1) and
robust (alpha 0) GNC stages.  CPU only.
usage: python tools/pair_block_iters.py H W"""
import sys, time, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'optical-flow-python_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT,'tools')]
import numpy as np, oracle as O
from scipy import sparse
from scipy.sparse.linalg import eigsh
from optical_flow.methods.config import load_of_method
from optical_flow.methods.base import planes_to_sparse
from optical_flow.utils.synthetic import synth_pair
H,W = int(sys.argv[1]), int(sys.argv[2])
im1, im2, gt = synth_pair(H, W, 0)
g = lambda im: np.floor(0.2989*im[...,0]+0.5870*im[...,1]+0.1140*im[...,2]+0.5)
imgs = np.stack([g(im1), g(im2)], 2)
tex = O.rof_texture(imgs)
o = load_of_method('classic+nl-fast')
uv = gt + 0.3*np.sin(np.arange(H)[:,None,None]/17.0)
It, Ix, Iy = O.partial_deriv(tex, uv, 'bi-cubic')
from numpy.polynomial import chebyshev as Ch, polynomial as Pl
def cheb(m, a, b=2.0):
    s=(b+a)/(b-a); gg=-2.0/(b-a)
    T=np.zeros(m+2); T[m+1]=1
    P=Ch.cheb2poly(T); Ts=np.polyval(P[::-1], s)
    R=np.zeros(1)
    for k,c in enumerate(P): R=Pl.polyadd(R, c*Pl.polypow([s,gg],k))
    R=R/Ts; pX=-R[1:]
    cB=np.zeros(m+1)
    for j,c in enumerate(pX): cB[:len(Pl.polypow([1,-1],j))]+=c*Pl.polypow([1,-1],j)
    return cB
n=H*W
idx = lambda i,j: j*H+i
for alpha in (1.0, 0.0):
    coef, rhs = O.flow_operator(o.to_params(), alpha, uv, None, It, Ix, Iy)
    A = planes_to_sparse(coef).tocsr()
    b = np.concatenate([rhs[0].ravel(order='F'), rhs[1].ravel(order='F')])
    a_, c_, d_ = coef[4].ravel(order='F'), coef[5].ravel(order='F'), coef[6].ravel(order='F')
    D = sparse.bmat([[sparse.diags(a_), sparse.diags(c_)],[sparse.diags(c_), sparse.diags(d_)]]).tocsr()
    # pair blocks: add the intra-pair edge (columns 2k, 2k+1) to D
    wxu = coef[0]; wxv = coef[2]   # weight of edge to the right, (H, W)
    I, J = np.meshgrid(np.arange(H), np.arange(0, W-1, 2), indexing='ij')
    r0 = idx(I, J).ravel(); r1 = idx(I, J+1).ravel()
    wu = wxu[I, J].ravel(); wv = wxv[I, J].ravel()
    rows = np.concatenate([r0, r1, r0+n, r1+n]); cols = np.concatenate([r1, r0, r1+n, r0+n])
    vals = -np.concatenate([wu, wu, wv, wv])
    Dp = (D + sparse.coo_matrix((vals, (rows, cols)), shape=(2*n, 2*n))).tocsc()
    Np = (Dp - A).tocsr()
    # inverse of block-diag Dp: factor with splu (exact, block-diagonal)
    from scipy.sparse.linalg import splu
    lu = splu(Dp)
    Dinv_apply = lambda r: lu.solve(r)
    det = a_*d_ - c_*c_
    Dinv = sparse.bmat([[sparse.diags(d_/det), sparse.diags(-c_/det)],[sparse.diags(-c_/det), sparse.diags(a_/det)]]).tocsr()
    N = (D - A).tocsr()
    for name, Di, NN in (('2x2', lambda r: Dinv @ r, N), ('pair4x4', Dinv_apply, Np)):
        # lambda_max of Di A (generalized): power iteration
        v = np.random.default_rng(0).standard_normal(2*n)
        for _ in range(60):
            v = Di(A @ v); lam = np.linalg.norm(v); v /= lam
        def pcg(m, lo, hi):
            cB = cheb(m, lo, hi)
            def Minv(r):
                y = Di(r); gg = cB[m]*y
                for i in range(m-1, -1, -1): gg = cB[i]*y + Di(NN @ gg)
                return gg
            x=np.zeros_like(b); r=b.copy(); z=Minv(r); p=z.copy(); rz=r@z; bn=np.linalg.norm(b)
            for k in range(3000):
                if np.linalg.norm(r) < 1e-6*bn: return k
                q=A@p; al=rz/(p@q); x+=al*p; r-=al*q; z=Minv(r); rz2=r@z; p=z+(rz2/rz)*p; rz=rz2
            return 3000
        for m in (5,):
            for lo in (0.01, 0.02, 0.04, 0.08):
                print(f'alpha {alpha} {name} lam_max~{lam:.4f} degree {m} lo {lo}: iters {pcg(m, lo, 2.0)}', flush=True)
