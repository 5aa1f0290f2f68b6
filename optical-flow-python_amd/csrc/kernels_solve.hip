// kernels_solve.hip — matrix-free iterative solvers for the 2N x 2N flow
// system (base.py:87-172): preconditioned CG with the exact control flow of
// scipy.sparse.linalg.cg (x0 = 0, stop when ||r|| < rtol ||b|| before an
// iteration, at most maxiter iterations), and red-black block SOR.
//
// One CG iteration = two launches (the two global reductions p.q and r.z
// are kernel boundaries): k_pcg_dir_spmv builds p = z + beta p_old on the fly,
// applies A and reduces p.q; k_pcg_update moves x and r, applies the
// preconditioner and reduces r.z and r.r.  The last block of each launch
// finishes the reduction in a fixed order (deterministic results) and
// updates the PcgState scalars; kernels of a converged solve exit at entry,
// so the host can enqueue iterations in chunks without waiting.
#include "kernels.h"

template <bool BLOCK>
__device__ __forceinline__ float2 precond(const float *__restrict__ coef, size_t ps, size_t k, float2 r) {
  const float a = coef[4 * ps + k], c = coef[5 * ps + k], d = coef[6 * ps + k];
  if (BLOCK) {
    const float det = a * d - c * c;
    if (det > 1e-30f * fabsf(a * d)) return make_float2((d * r.x - c * r.y) / det, (a * r.y - c * r.x) / det);
  }
  // scalar Jacobi, base.py:129-131: 1/diag where |diag| > 1e-12 else 0
  return make_float2(fabsf(a) > 1e-12f ? r.x / a : 0.0f, fabsf(d) > 1e-12f ? r.y / d : 0.0f);
}

__device__ __forceinline__ void finish_state_init(PcgState *st, double rz, double rr, double rtol, int maxiter) {
  st->rho = rz;
  st->rr = rr;
  st->bnorm = sqrt(rr);
  st->atol = rtol * st->bnorm;
  st->iter = 0;
  st->maxiter = maxiter;
  st->alpha = 0.0f;
  st->beta = 0.0f;
  st->done = st->bnorm == 0.0 ? 3 : (sqrt(rr) < st->atol ? 1 : (maxiter <= 0 ? 2 : 0));
}

// x = 0, r = b, z = M^-1 b; reduce r.z, r.r
template <bool BLOCK>
__global__ void k_pcg_init(const float *__restrict__ coef, const float2 *__restrict__ b, float2 *__restrict__ x,
                           float2 *__restrict__ r, float2 *__restrict__ z, int H, int W, int P, size_t ps,
                           PcgState *st, double *partials, unsigned *counter, double rtol, int maxiter) {
  __shared__ double lds[32];
  double v[2] = {0.0, 0.0};
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    const float2 bb = b[k];
    const float2 zz = precond<BLOCK>(coef, ps, k, bb);
    x[k] = make_float2(0.0f, 0.0f);
    r[k] = bb;
    z[k] = zz;
    v[0] += (double)bb.x * zz.x + (double)bb.y * zz.y;
    v[1] += (double)bb.x * bb.x + (double)bb.y * bb.y;
  }
  block_sum<2>(v, lds);
  const int nb = gridDim.x * gridDim.y;
  if (arrive_last<2>(v, partials, counter, nb, blockIdx.x + blockIdx.y * gridDim.x)) {
    double s[2];
    final_sum<2>(s, partials, nb, lds);
    if (threadIdx.x == 0 && threadIdx.y == 0) {
      finish_state_init(st, s[0], s[1], rtol, maxiter);
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// p_new = z + beta p_old (p = z on the first iteration), q = A p_new, reduce p.q
__global__ void k_pcg_dir_spmv(const float *__restrict__ coef, const float2 *__restrict__ z,
                               const float2 *__restrict__ pold, float2 *__restrict__ pnew, float2 *__restrict__ q,
                               int H, int W, int P, size_t ps, PcgState *st, double *partials, unsigned *counter) {
  if (st->done) return;
  __shared__ double lds[16];
  const bool first = st->iter == 0;
  const float beta = st->beta;
  auto pn = [&](size_t kk) -> float2 {
    float2 a = z[kk];
    if (!first) {
      const float2 b = pold[kk];
      a.x += beta * b.x;
      a.y += beta * b.y;
    }
    return a;
  };
  double v[1] = {0.0};
  const float *wxu = coef, *wyu = coef + ps, *wxv = coef + 2 * ps, *wyv = coef + 3 * ps;
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    const float2 c = pn(k);
    pnew[k] = c;
    float su = 0.0f, sv = 0.0f;
    if (j < W - 1) { const float2 n = pn(k + 1); su += wxu[k] * n.x; sv += wxv[k] * n.y; }
    if (j > 0) { const float2 n = pn(k - 1); su += wxu[k - 1] * n.x; sv += wxv[k - 1] * n.y; }
    if (i < H - 1) { const float2 n = pn(k + P); su += wyu[k] * n.x; sv += wyv[k] * n.y; }
    if (i > 0) { const float2 n = pn(k - P); su += wyu[k - P] * n.x; sv += wyv[k - P] * n.y; }
    const float a = coef[4 * ps + k], cc = coef[5 * ps + k], d = coef[6 * ps + k];
    const float2 qq = make_float2(a * c.x + cc * c.y - su, cc * c.x + d * c.y - sv);
    q[k] = qq;
    v[0] += (double)c.x * qq.x + (double)c.y * qq.y;
  }
  block_sum<1>(v, lds);
  const int nb = gridDim.x * gridDim.y;
  if (arrive_last<1>(v, partials, counter, nb, blockIdx.x + blockIdx.y * gridDim.x)) {
    double s[1];
    final_sum<1>(s, partials, nb, lds);
    if (threadIdx.x == 0 && threadIdx.y == 0) {
      st->pq = s[0];
      st->alpha = (float)(st->rho / s[0]);
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// x += alpha p, r -= alpha q, z = M^-1 r; reduce r.z, r.r; convergence test
template <bool BLOCK>
__global__ void k_pcg_update(const float *__restrict__ coef, float2 *__restrict__ x, float2 *__restrict__ r,
                             const float2 *__restrict__ p, const float2 *__restrict__ q, float2 *__restrict__ z, int H,
                             int W, int P, size_t ps, PcgState *st, double *partials, unsigned *counter) {
  if (st->done) return;
  __shared__ double lds[32];
  const float alpha = st->alpha;
  double v[2] = {0.0, 0.0};
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    const float2 pp = p[k], qq = q[k];
    float2 xx = x[k], rr = r[k];
    xx.x += alpha * pp.x;
    xx.y += alpha * pp.y;
    rr.x -= alpha * qq.x;
    rr.y -= alpha * qq.y;
    x[k] = xx;
    r[k] = rr;
    const float2 zz = precond<BLOCK>(coef, ps, k, rr);
    z[k] = zz;
    v[0] += (double)rr.x * zz.x + (double)rr.y * zz.y;
    v[1] += (double)rr.x * rr.x + (double)rr.y * rr.y;
  }
  block_sum<2>(v, lds);
  const int nb = gridDim.x * gridDim.y;
  if (arrive_last<2>(v, partials, counter, nb, blockIdx.x + blockIdx.y * gridDim.x)) {
    double s[2];
    final_sum<2>(s, partials, nb, lds);
    if (threadIdx.x == 0 && threadIdx.y == 0) {
      const double rho_new = s[0];
      st->beta = (float)(rho_new / st->rho);
      st->rho = rho_new;
      st->rr = s[1];
      st->iter += 1;
      if (sqrt(s[1]) < st->atol) st->done = 1;
      else if (st->iter >= st->maxiter) st->done = 2;
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------
// red-black block SOR (the GPU form of base.py:138-172): pixels of one colour
// are independent; each solves its own 2x2 (u, v) block against the current
// neighbours and relaxes with omega.  Convergence: ||x - x_old|| < tol ||x||
// per full sweep (red + black), evaluated in the black pass's last block.
__global__ void k_sor_init(float2 *x, int H, int W, int P, PcgState *st, int maxiter) {
  OF_FOR_PIXELS(H, W) {
    if (j < W) x[(size_t)i * P + j] = make_float2(0.0f, 0.0f);
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && threadIdx.y == 0) {
    st->iter = 0;
    st->maxiter = maxiter;
    st->done = maxiter <= 0 ? 2 : 0;
    st->xnorm2 = st->dnorm2 = 0.0;
  }
}

__global__ void k_sor_sweep(const float *__restrict__ coef, const float2 *__restrict__ b, float2 *__restrict__ x,
                            int H, int W, int P, size_t ps, int color, float omega, float tol, PcgState *st,
                            double *partials, unsigned *counter) {
  if (st->done) return;
  __shared__ double lds[32];
  double v[2] = {0.0, 0.0};
  const float *wxu = coef, *wyu = coef + ps, *wxv = coef + 2 * ps, *wyv = coef + 3 * ps;
  OF_FOR_PIXELS(H, W) {
    if (j >= W || ((i + j) & 1) != color) continue;
    const size_t k = (size_t)i * P + j;
    float2 s = b[k];
    if (j < W - 1) { const float2 n = x[k + 1]; s.x += wxu[k] * n.x; s.y += wxv[k] * n.y; }
    if (j > 0) { const float2 n = x[k - 1]; s.x += wxu[k - 1] * n.x; s.y += wxv[k - 1] * n.y; }
    if (i < H - 1) { const float2 n = x[k + P]; s.x += wyu[k] * n.x; s.y += wyv[k] * n.y; }
    if (i > 0) { const float2 n = x[k - P]; s.x += wyu[k - P] * n.x; s.y += wyv[k - P] * n.y; }
    const float a = coef[4 * ps + k], c = coef[5 * ps + k], d = coef[6 * ps + k];
    const float det = a * d - c * c;
    float2 y;
    if (det > 1e-30f * fabsf(a * d)) y = make_float2((d * s.x - c * s.y) / det, (a * s.y - c * s.x) / det);
    else y = make_float2(fabsf(a) > 1e-15f ? s.x / a : 0.0f, fabsf(d) > 1e-15f ? s.y / d : 0.0f);
    const float2 o = x[k];
    const float2 nw = make_float2(o.x + omega * (y.x - o.x), o.y + omega * (y.y - o.y));
    x[k] = nw;
    v[0] += (double)(nw.x - o.x) * (nw.x - o.x) + (double)(nw.y - o.y) * (nw.y - o.y);
    v[1] += (double)nw.x * nw.x + (double)nw.y * nw.y;
  }
  block_sum<2>(v, lds);
  const int nb = gridDim.x * gridDim.y;
  if (arrive_last<2>(v, partials, counter, nb, blockIdx.x + blockIdx.y * gridDim.x)) {
    double s[2];
    final_sum<2>(s, partials, nb, lds);
    if (threadIdx.x == 0 && threadIdx.y == 0) {
      if (color == 0) {
        st->dnorm2 = s[0];
        st->xnorm2 = s[1];
      } else {
        const double dn = st->dnorm2 + s[0], xn = st->xnorm2 + s[1];
        st->iter += 1;
        st->rr = dn;
        if (sqrt(dn) < (double)tol * sqrt(xn)) st->done = 1;
        else if (st->iter >= st->maxiter) st->done = 2;
      }
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
