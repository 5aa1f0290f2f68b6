// kernels_solve.hip — matrix-free iterative solvers for the 2N x 2N flow
// system (base.py:87-172): preconditioned CG with the exact control flow of
// scipy.sparse.linalg.cg (x0 = 0, stop when ||r|| < rtol ||b|| before an
// iteration, at most maxiter iterations), and red-black block SOR.
//
// One CG iteration = two launches; each global reduction is finished in the
// PROLOGUE of the next launch (the launch-boundary reduce): every block of
// the consumer sums the producer's per-block partials in the same fixed
// order, so all blocks derive bit-identical scalars and no agent-scope
// fence or atomic is needed (kernel boundaries give visibility).
//
//   spmv(k)   prologue: (k > 0) rz, rr of update(k-1) -> convergence test,
//             beta = rz / rho[k-1]; body: p = z + beta p_old, q = A p,
//             per-block p.q
//   update(k) prologue: pq of spmv(k) -> alpha = rho[k] / pq; body:
//             x += alpha p, r -= alpha q, z = M^-1 r, per-block r.z, r.r
//
// Kernels of a finished solve return at entry, so the host can enqueue
// iterations in chunks.  Each thread owns two horizontally adjacent pixels
// (8-B loads of scalar planes, 16-B loads of float2 fields).
#include "kernels.h"

#define PCG_MAX_BLOCKS 512

template <bool BLOCK>
__device__ __forceinline__ float2 precond(float a, float c, float d, float2 r) {
  if (BLOCK) {
    const float det = a * d - c * c;
    if (det > 1e-30f * fabsf(a * d)) {
      const float inv = 1.0f / det;
      return make_float2((d * r.x - c * r.y) * inv, (a * r.y - c * r.x) * inv);
    }
  }
  // scalar Jacobi, base.py:129-131: 1/diag where |diag| > 1e-12 else 0
  return make_float2(fabsf(a) > 1e-12f ? r.x / a : 0.0f, fabsf(d) > 1e-12f ? r.y / d : 0.0f);
}

// fixed-order sum of NV partial arrays (stride nb) by the whole block;
// result broadcast to every thread
template <int NV>
__device__ __forceinline__ void prologue_sum(double (&out)[NV], const double *__restrict__ part, int nb, double *lds) {
  const int tid = threadIdx.x + threadIdx.y * blockDim.x, nt = blockDim.x * blockDim.y;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    double s = 0.0;
    for (int b = tid; b < nb; b += nt) s += part[(size_t)v * PCG_MAX_BLOCKS + b];
    out[v] = wave_sum(s);
  }
  if ((tid & 63) == 0)
#pragma unroll
    for (int v = 0; v < NV; ++v) lds[v * 8 + (tid >> 6)] = out[v];
  __syncthreads();
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    double s = 0.0;
    for (int w = 0; w < nt / 64; ++w) s += lds[v * 8 + w];
    out[v] = s;
  }
  __syncthreads();
}

// per-block partials -> part[v * PCG_MAX_BLOCKS + bid] (plain stores)
template <int NV>
__device__ __forceinline__ void write_partials(double (&v)[NV], double *part, double *lds) {
  const int tid = threadIdx.x + threadIdx.y * blockDim.x, nt = blockDim.x * blockDim.y;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
  if ((tid & 63) == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) lds[k * 8 + (tid >> 6)] = v[k];
  __syncthreads();
  if (tid == 0) {
    const int bid = blockIdx.x + blockIdx.y * gridDim.x;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double s = 0.0;
      for (int w = 0; w < nt / 64; ++w) s += lds[k * 8 + w];
      part[(size_t)k * PCG_MAX_BLOCKS + bid] = s;
    }
  }
}

// two-pixel loop: thread (tx, ty) of block (bx, by) owns columns
// j0 = 2 * (bx * 64 + tx), j0 + 1 of rows by*4+ty, + gridDim.y*4, ...
#define OF_FOR_PIXEL_PAIRS(H, W)                                         \
  const int j0 = 2 * (blockIdx.x * OF_BX + threadIdx.x);                 \
  for (int i = blockIdx.y * OF_BY + threadIdx.y; i < (H); i += gridDim.y * OF_BY)

struct PcgArgs {
  const float *coef;  // 7 planes, plane stride ps
  float2 *x, *r, *z, *p_old, *p_new, *q;
  const float2 *b;
  int H, W, P;
  size_t ps;
  int nb;  // blocks of this grid (== blocks of every launch of the solve)
  double *part;  // [3][PCG_MAX_BLOCKS]: 0 = p.q, 1 = r.z, 2 = r.r
  PcgState *st;
  double rtol;
  int maxiter;
};

// x = 0, r = b, z = M^-1 b; partials r.z, r.r
template <bool BLOCK>
__global__ __launch_bounds__(256) void k_pcg_init(PcgArgs a) {
  __shared__ double lds[32];
  double v[2] = {0.0, 0.0};
  const float *A = a.coef + 4 * a.ps, *Cc = a.coef + 5 * a.ps, *D = a.coef + 6 * a.ps;
  OF_FOR_PIXEL_PAIRS(a.H, a.W) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = j0 + e;
      if (j >= a.W) break;
      const size_t k = (size_t)i * a.P + j;
      const float2 bb = a.b[k];
      const float2 zz = precond<BLOCK>(A[k], Cc[k], D[k], bb);
      a.x[k] = make_float2(0.0f, 0.0f);
      a.r[k] = bb;
      a.z[k] = zz;
      v[0] += (double)bb.x * zz.x + (double)bb.y * zz.y;
      v[1] += (double)bb.x * bb.x + (double)bb.y * bb.y;
    }
  }
  write_partials<2>(v, a.part + PCG_MAX_BLOCKS, lds);
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && threadIdx.y == 0) {
    a.st->done = a.maxiter <= 0 ? 2 : 0;
    a.st->iter = 0;
    a.st->maxiter = a.maxiter;
  }
}

__device__ __forceinline__ float2 lin(float2 z, float2 p, float beta) {
  return make_float2(z.x + beta * p.x, z.y + beta * p.y);
}

// p_new = z + beta p_old (p = z when k == 0), q = A p_new; partial p.q
__global__ __launch_bounds__(256) void k_pcg_dir_spmv(PcgArgs a, int k) {
  __shared__ double lds[32];
  __shared__ int s_exit;
  if (a.st->done) return;
  double sums[2];
  prologue_sum<2>(sums, a.part + PCG_MAX_BLOCKS, a.nb, lds);  // r.z, r.r of update(k-1) / init
  const bool lead = blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && threadIdx.y == 0;
  double beta_d = 0.0;
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    int done = 0;
    double atol;
    if (k == 0) {
      const double bn = sqrt(sums[1]);
      atol = a.rtol * bn;
      if (lead) { a.st->bnorm = bn; a.st->atol = atol; }
      if (bn == 0.0) done = 3;
    } else {
      atol = a.st->atol;
      beta_d = sums[0] / a.st->rho[(k - 1) & 1];
    }
    if (!done && sqrt(sums[1]) < atol) done = 1;  // scipy cg: check before the iteration
    if (!done && k >= a.maxiter) done = 2;
    if (lead) {
      a.st->rho[k & 1] = sums[0];
      a.st->rr = sums[1];
      a.st->iter = k;
      if (done) a.st->done = done;
    }
    s_exit = done;
    lds[31] = beta_d;
  }
  __syncthreads();
  if (s_exit) return;
  const float beta = (float)lds[31];
  const bool first = k == 0;
  const float *wxu = a.coef, *wyu = a.coef + a.ps, *wxv = a.coef + 2 * a.ps, *wyv = a.coef + 3 * a.ps;
  const float *A = a.coef + 4 * a.ps, *Cc = a.coef + 5 * a.ps, *D = a.coef + 6 * a.ps;
  const int H = a.H, W = a.W, P = a.P;
  double v[1] = {0.0};
  OF_FOR_PIXEL_PAIRS(H, W) {
    if (j0 >= W) continue;
    const size_t k0 = (size_t)i * P + j0;
    const bool two = j0 + 1 < W;
    // p at this pair and its 4-neighbourhood
    auto pn = [&](size_t kk) -> float2 { return first ? a.z[kk] : lin(a.z[kk], a.p_old[kk], beta); };
    const float2 c0 = pn(k0), c1 = two ? pn(k0 + 1) : make_float2(0.f, 0.f);
    const float2 l0 = j0 > 0 ? pn(k0 - 1) : make_float2(0.f, 0.f);
    const float2 r1 = j0 + 2 < W ? pn(k0 + 2) : make_float2(0.f, 0.f);
    a.p_new[k0] = c0;
    if (two) a.p_new[k0 + 1] = c1;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if (e == 1 && !two) break;
      const int j = j0 + e;
      const size_t kk = k0 + e;
      const float2 c = e ? c1 : c0;
      const float2 L = e ? c0 : l0, R = e ? r1 : c1;
      float su = 0.0f, sv = 0.0f;
      if (j < W - 1) { su += wxu[kk] * R.x; sv += wxv[kk] * R.y; }
      if (j > 0) { su += wxu[kk - 1] * L.x; sv += wxv[kk - 1] * L.y; }
      if (i < H - 1) { const float2 n = pn(kk + P); su += wyu[kk] * n.x; sv += wyv[kk] * n.y; }
      if (i > 0) { const float2 n = pn(kk - P); su += wyu[kk - P] * n.x; sv += wyv[kk - P] * n.y; }
      const float aa = A[kk], cc = Cc[kk], dd = D[kk];
      const float2 qq = make_float2(aa * c.x + cc * c.y - su, cc * c.x + dd * c.y - sv);
      a.q[kk] = qq;
      v[0] += (double)c.x * qq.x + (double)c.y * qq.y;
    }
  }
  write_partials<1>(v, a.part, lds);
}

// x += alpha p, r -= alpha q, z = M^-1 r; partials r.z, r.r
template <bool BLOCK>
__global__ __launch_bounds__(256) void k_pcg_update(PcgArgs a, int k) {
  __shared__ double lds[32];
  if (a.st->done) return;
  double pq[1];
  prologue_sum<1>(pq, a.part, a.nb, lds);
  const float alpha = (float)(a.st->rho[k & 1] / pq[0]);
  const float *A = a.coef + 4 * a.ps, *Cc = a.coef + 5 * a.ps, *D = a.coef + 6 * a.ps;
  double v[2] = {0.0, 0.0};
  OF_FOR_PIXEL_PAIRS(a.H, a.W) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = j0 + e;
      if (j >= a.W) break;
      const size_t kk = (size_t)i * a.P + j;
      const float2 pp = a.p_new[kk], qq = a.q[kk];
      float2 xx = a.x[kk], rr = a.r[kk];
      xx.x += alpha * pp.x;
      xx.y += alpha * pp.y;
      rr.x -= alpha * qq.x;
      rr.y -= alpha * qq.y;
      a.x[kk] = xx;
      a.r[kk] = rr;
      const float2 zz = precond<BLOCK>(A[kk], Cc[kk], D[kk], rr);
      a.z[kk] = zz;
      v[0] += (double)rr.x * zz.x + (double)rr.y * zz.y;
      v[1] += (double)rr.x * rr.x + (double)rr.y * rr.y;
    }
  }
  write_partials<2>(v, a.part + PCG_MAX_BLOCKS, lds);
}

// after the last enqueued iteration: record the final state for the host
__global__ __launch_bounds__(256) void k_pcg_final(PcgArgs a, int k) {
  __shared__ double lds[32];
  if (a.st->done) return;
  double sums[2];
  prologue_sum<2>(sums, a.part + PCG_MAX_BLOCKS, a.nb, lds);
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    a.st->rr = sums[1];
    a.st->iter = k;
    a.st->done = sqrt(sums[1]) < a.st->atol ? 1 : 2;
  }
}

// ---------------------------------------------------------------------------
// red-black block SOR (the GPU form of base.py:138-172): pixels of one colour
// are independent; each solves its own 2x2 (u, v) block against the current
// neighbours and relaxes with omega.  Convergence ||x - x_old|| < tol ||x||
// per full sweep is evaluated in the prologue of the next red sweep.
struct SorArgs {
  const float *coef;
  const float2 *b;
  float2 *x;
  int H, W, P;
  size_t ps;
  int nb;
  double *part;  // [2 colours][2 sums][PCG_MAX_BLOCKS]
  PcgState *st;
  float omega, tol;
  int maxiter;
};

__global__ __launch_bounds__(256) void k_sor_init(SorArgs a) {
  OF_FOR_PIXELS(a.H, a.W) {
    if (j < a.W) a.x[(size_t)i * a.P + j] = make_float2(0.0f, 0.0f);
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && threadIdx.y == 0) {
    a.st->iter = 0;
    a.st->maxiter = a.maxiter;
    a.st->done = a.maxiter <= 0 ? 2 : 0;
  }
}

__global__ __launch_bounds__(256) void k_sor_sweep(SorArgs a, int color, int k) {
  __shared__ double lds[32];
  __shared__ int s_exit;
  if (a.st->done) return;
  if (color == 0 && k > 0) {
    double s[4];
    prologue_sum<4>(s, a.part, a.nb, lds);  // red dn, red xn, black dn, black xn of sweep k-1
    if (threadIdx.x == 0 && threadIdx.y == 0) {
      const double dn = s[0] + s[2], xn = s[1] + s[3];
      int done = sqrt(dn) < (double)a.tol * sqrt(xn) ? 1 : (k >= a.maxiter ? 2 : 0);
      if (blockIdx.x == 0 && blockIdx.y == 0) {
        a.st->iter = k;
        a.st->rr = dn;
        if (done) a.st->done = done;
      }
      s_exit = done;
    }
    __syncthreads();
    if (s_exit) return;
  }
  double v[2] = {0.0, 0.0};
  const float *wxu = a.coef, *wyu = a.coef + a.ps, *wxv = a.coef + 2 * a.ps, *wyv = a.coef + 3 * a.ps;
  OF_FOR_PIXELS(a.H, a.W) {
    if (j >= a.W || ((i + j) & 1) != color) continue;
    const int W = a.W, H = a.H, P = a.P;
    const size_t kk = (size_t)i * P + j;
    float2 s = a.b[kk];
    if (j < W - 1) { const float2 n = a.x[kk + 1]; s.x += wxu[kk] * n.x; s.y += wxv[kk] * n.y; }
    if (j > 0) { const float2 n = a.x[kk - 1]; s.x += wxu[kk - 1] * n.x; s.y += wxv[kk - 1] * n.y; }
    if (i < H - 1) { const float2 n = a.x[kk + P]; s.x += wyu[kk] * n.x; s.y += wyv[kk] * n.y; }
    if (i > 0) { const float2 n = a.x[kk - P]; s.x += wyu[kk - P] * n.x; s.y += wyv[kk - P] * n.y; }
    const float aa = a.coef[4 * a.ps + kk], c = a.coef[5 * a.ps + kk], d = a.coef[6 * a.ps + kk];
    const float det = aa * d - c * c;
    float2 y;
    if (det > 1e-30f * fabsf(aa * d)) y = make_float2((d * s.x - c * s.y) / det, (aa * s.y - c * s.x) / det);
    else y = make_float2(fabsf(aa) > 1e-15f ? s.x / aa : 0.0f, fabsf(d) > 1e-15f ? s.y / d : 0.0f);
    const float2 o = a.x[kk];
    const float2 nw = make_float2(o.x + a.omega * (y.x - o.x), o.y + a.omega * (y.y - o.y));
    a.x[kk] = nw;
    v[0] += (double)(nw.x - o.x) * (nw.x - o.x) + (double)(nw.y - o.y) * (nw.y - o.y);
    v[1] += (double)nw.x * nw.x + (double)nw.y * nw.y;
  }
  write_partials<2>(v, a.part + (size_t)color * 2 * PCG_MAX_BLOCKS, lds);
}

__global__ __launch_bounds__(256) void k_sor_final(SorArgs a, int k) {
  __shared__ double lds[32];
  if (a.st->done) return;
  double s[4];
  prologue_sum<4>(s, a.part, a.nb, lds);
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    const double dn = s[0] + s[2], xn = s[1] + s[3];
    a.st->iter = k;
    a.st->rr = dn;
    a.st->done = sqrt(dn) < (double)a.tol * sqrt(xn) ? 1 : 2;
  }
}

// ---------------------------------------------------------------------------
// sum of squares of a float2 field (HS early exit ||x||_2 < 1e-3, hs.py:127):
// partials then a one-block finish
__global__ __launch_bounds__(256) void k_norm2_part(const float2 *__restrict__ x, int H, int W, int P, double *part) {
  __shared__ double lds[32];
  double v[1] = {0.0};
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const float2 a = x[(size_t)i * P + j];
    v[0] += (double)a.x * a.x + (double)a.y * a.y;
  }
  write_partials<1>(v, part, lds);
}
__global__ __launch_bounds__(256) void k_norm2_final(const double *part, int nb, double *result) {
  __shared__ double lds[32];
  double s[1];
  prologue_sum<1>(s, part, nb, lds);
  if (threadIdx.x == 0 && threadIdx.y == 0) *result = s[0];
}
