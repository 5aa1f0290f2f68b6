"""Degree-5 polynomial preconditioners p(B) D^-1 for the robust stage: the
production Chebyshev minimax on [a, 2] vs least-squares polynomials (min of
the weighted L2 norm of 1 - X p(X) over [a, 2]), CG iterations to 1e-6 on the
oracle-assembled 540x960 Classic+NL-fast operator (tools/poly_iters.py).
usage: python tools/poly_alt.py [H W]"""
import sys, os, time
ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'optical-flow-python_amd'), os.path.join(ROOT, 'oracle'), os.path.join(ROOT,'tools')]
import numpy as np, oracle as O
from scipy import sparse
from numpy.polynomial import polynomial as Pl
from optical_flow.methods.config import load_of_method
from optical_flow.methods.base import planes_to_sparse
from optical_flow.utils.synthetic import synth_pair
H,W = int(sys.argv[1]) if len(sys.argv)>1 else 540, int(sys.argv[2]) if len(sys.argv)>2 else 960
im1, im2, gt = synth_pair(H, W, 0)
g = lambda im: np.floor(0.2989*im[...,0]+0.5870*im[...,1]+0.1140*im[...,2]+0.5)
imgs = np.stack([g(im1), g(im2)], 2)
tex = O.rof_texture(imgs)
o = load_of_method('classic+nl-fast')
uv = gt + 0.3*np.sin(np.arange(H)[:,None,None]/17.0)
It, Ix, Iy = O.partial_deriv(tex, uv, 'bi-cubic')

def to_B(pX):
    m=len(pX)-1; cB=np.zeros(m+1)
    for j,c in enumerate(pX):
        q=Pl.polypow([1,-1],j); cB[:len(q)]+=c*q
    return cB
def cheb(m, a, b=2.0):
    from numpy.polynomial import chebyshev as Ch
    s=(b+a)/(b-a); gg=-2.0/(b-a)
    T=np.zeros(m+2); T[m+1]=1
    P=Ch.cheb2poly(T); Ts=np.polyval(P[::-1], s)
    R=np.zeros(1)
    for k,c in enumerate(P): R=Pl.polyadd(R, c*Pl.polypow([s,gg],k))
    R=R/Ts
    return -R[1:]
def lsq(m, a, b=2.0, weight='cheb', n=4000):
    # minimise sum w(x) (1 - x p(x))^2 over nodes in [a, b]
    if weight=='cheb':
        t=np.cos(np.pi*(np.arange(n)+0.5)/n); x=(a+b)/2+(b-a)/2*t; w=np.ones(n)
    else:
        x=np.linspace(a,b,n); w=np.ones(n)
        if weight=='x': w=x
    V=np.stack([x**(k+1) for k in range(m+1)],1)
    c,*_=np.linalg.lstsq(V*np.sqrt(w)[:,None], np.sqrt(w), rcond=None)
    return c
alpha=0.0
coef, rhs = O.flow_operator(o.to_params(), alpha, uv, None, It, Ix, Iy)
A = planes_to_sparse(coef).tocsr()
b = np.concatenate([rhs[0].ravel(order='F'), rhs[1].ravel(order='F')])
a_, c_, d_ = coef[4].ravel(order='F'), coef[5].ravel(order='F'), coef[6].ravel(order='F')
det = a_*d_ - c_*c_
Dinv = sparse.bmat([[sparse.diags(d_/det), sparse.diags(-c_/det)],[sparse.diags(-c_/det), sparse.diags(a_/det)]]).tocsr()
D = sparse.bmat([[sparse.diags(a_), sparse.diags(c_)],[sparse.diags(c_), sparse.diags(d_)]]).tocsr()
B = (Dinv @ (D - A)).tocsr()
def pcg(cB):
    m=len(cB)-1
    def Minv(r):
        y = Dinv @ r; gq = cB[m]*y
        for i in range(m-1, -1, -1): gq = cB[i]*y + B @ gq
        return gq
    x=np.zeros_like(b); r=b.copy(); z=Minv(r); p=z.copy(); rz=r@z; bn=np.linalg.norm(b)
    for k in range(3000):
        if np.linalg.norm(r) < 1e-6*bn: return k
        q=A@p; al=rz/(p@q); x+=al*p; r-=al*q; z=Minv(r); rz2=r@z
        if rz2<=0: return -k
        p=z+(rz2/rz)*p; rz=rz2
    return 3000
xs=np.linspace(1e-4,2,20001)
for name, pX in [('cheb a=0.02', cheb(5,0.02)), ('cheb a=0.04', cheb(5,0.04)), ('cheb a=0.01', cheb(5,0.01)),
                 ('lsq-cheb a=0.0', lsq(5,0.0)), ('lsq-cheb a=0.01', lsq(5,0.01)), ('lsq-cheb a=0.02', lsq(5,0.02)),
                 ('lsq-unif a=0', lsq(5,0.0,weight='unif')), ('lsq-x a=0', lsq(5,0.0,weight='x'))]:
    pv=np.polyval(pX[::-1], xs); ok=pv.min()>0
    print(f'{name:18s} p>0 on (0,2]: {ok}  min p {pv.min():.3g}  max|1-xp| on [0.02,2] {np.abs(1-xs*pv)[xs>=0.02].max():.3f}  iters {pcg(to_B(pX))}', flush=True)
