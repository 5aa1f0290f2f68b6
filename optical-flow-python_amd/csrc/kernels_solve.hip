// kernels_solve.hip — matrix-free iterative solvers for the 2N x 2N flow
// system (base.py:87-172): preconditioned CG with the exact control flow of
// scipy.sparse.linalg.cg (x0 = 0, stop when ||r|| < rtol ||b|| before an
// iteration, at most maxiter iterations), and red-black block SOR.
//
// CG: ONE launch per iteration (k_cg, below).  Every global reduction is
// finished in the PROLOGUE of the next launch (launch-boundary reduce): each
// block of the consumer sums the producer's per-block partials in the same
// fixed order, so all blocks derive bit-identical scalars, and no
// agent-scope fence or atomic is needed (kernel boundaries give visibility).
// Launches of a finished solve return after the prologue, so the host can
// enqueue iterations in chunks and poll a pinned status word.
#include "kernels.h"

#define PCG_MAX_BLOCKS 512
// degree of the Chebyshev polynomial preconditioner of the 'backslash'
// surrogate (k_cgs, k_cg_small): 5 needs 0.70x the iterations of 3 on
// Classic+NL stage-2 systems (tools/poly_iters.py), and its two extra stencil
// stages run on the two waves of a k_cgs block that had idle time
#define CG_DEG 5

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
__device__ __forceinline__ void write_partials(double (&v)[NV], double *part, double *lds, int slot = -1) {
  const int tid = threadIdx.x + threadIdx.y * blockDim.x, nt = blockDim.x * blockDim.y;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
  if ((tid & 63) == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) lds[k * 8 + (tid >> 6)] = v[k];
  __syncthreads();
  if (tid == 0) {
    const int bid = slot >= 0 ? slot : blockIdx.x + blockIdx.y * gridDim.x;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double s = 0.0;
      for (int w = 0; w < nt / 64; ++w) s += lds[k * 8 + w];
      part[(size_t)k * PCG_MAX_BLOCKS + bid] = s;
    }
  }
}

struct PcgArgs {
  const float *coef;  // 7 planes, plane stride ps
  float2 *x;
  const float2 *r_in, *p_old;  // iterate k-1
  float2 *r_out, *p_new;       // iterate k
  const float2 *b;
  int H, W, P;
  size_t ps;
  int nb;  // blocks of this grid (== blocks of every launch of the solve)
  // per-block partial sums [5][PCG_MAX_BLOCKS], ping-ponged by iteration
  // parity: launch k reads launch k-1's (part_rd) and writes its own
  // (part_wr).  One buffer would race: a block that starts after another
  // block of the same grid has finished would read a mix of both launches.
  const double *part_rd;
  double *part_wr;
  PcgState *st;
  CgFlag *hflag;  // mapped host memory (may be null)
  double rtol;
  int maxiter;
  float poly[8];  // k_cgs: M^-1 = (poly[0] + poly[1] B + ... + poly[CG_DEG] B^CG_DEG) D^-1
  // 'backslash' residual replacement (k_cg_update; null / 0 for 'pcg'):
  // x_hi (the iterate at the replacement) and the relative residual at which
  // it acts
  float2 *xh;
  double upd_rel;
};

// the shared prologue: returns 1 when the solve is finished (state written)
__device__ __forceinline__ int pcg_prologue(const PcgArgs &g, int k, double *lds, float *alpha, float *beta) {
  __shared__ int s_exit;
  __shared__ float s_ab[2];
  double S[5];
  prologue_sum<5>(S, g.part_rd, g.nb, lds);  // of K_{k-1}: pq, qz, qMq, rz, rr
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    const bool lead = blockIdx.x == 0 && blockIdx.y == 0;
    const double rn = sqrt(S[4]);
    const double atol = k == 1 ? g.rtol * rn : g.st->atol;
    int done = 0;
    if (k == 1 && S[4] == 0.0) done = 3;
    else if (rn < atol || S[4] == 0.0) done = 1;  // exact solution: nothing left to divide
    const double al = S[3] / S[0];
    const double rho = S[3] - 2.0 * al * S[1] + al * al * S[2];
    if (!done && (!(S[0] > 0.0) || !(S[3] > 0.0) || !(rho > 0.0))) done = 1;  // noise floor (cg_prologue)
    else if (!done && k - 1 >= g.maxiter) done = 2;
    if (lead) {
      if (k == 1) { g.st->bnorm = rn; g.st->atol = atol; }
      g.st->iter = k - 1;
      g.st->rr = S[4];
      g.st->rho[k & 1] = rho;
      if (done) g.st->done = done;
    }
    s_exit = done;
    s_ab[0] = (float)al;
    s_ab[1] = (float)(rho / S[3]);
  }
  __syncthreads();
  *alpha = s_ab[0];
  *beta = s_ab[1];
  return s_exit;
}

// ---------------------------------------------------------------------------
// q-free fused CG iteration on raw buffer loads (k_cg): the production CG
// kernel.  Same algebra as k_pcg_iter (rho recurrence, launch-boundary
// reduction), but
//  - q_{k-1} = A p_{k-1} is recomputed from p_{k-1} (read anyway, 2-row
//    halo) instead of being stored and re-read: 76 B/px per iteration
//    (r, x read+write; p_old read; p_new write; 7 coefficient planes);
//  - every load is a raw buffer load whose out-of-image offsets (rows outside
//    [0, H), columns outside [0, W)) return 0 by the hardware range check, so
//    the stencil needs no boundary branches, and stores from halo lanes are
//    dropped the same way;
//  - the first iteration and the 2x2 block / scalar Jacobi choice are
//    template parameters; dot products are formed per lane in fp32 over the
//    lane's two pixels and accumulated in fp64;
//  - the launch prologue issues the partial-sum loads, the state loads and
//    the first pipeline rows together (one memory round trip, not four).
// Geometry: a wave owns PCG_SW = 124 output columns; lane l holds columns
// jc = j0 - 2 + 2l and jc + 1, so lanes 0 and 63 carry the strip halo and all
// horizontal neighbours are DPP wave shifts.  A band of R rows is swept top
// to bottom; step t prefetches row t+1 (coefficients, r_in) and p_old of row
// t+2, forms r, z, p of row t and finishes row t-1 (q = A p, stores, dots).
#define PCG_SW 124
#define CG_OOB 0x80000000u

typedef float cg_f2 __attribute__((ext_vector_type(2)));
typedef float cg_f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t cg_rsrc(const void *p, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)min(bytes, (size_t)0x7fffffff), 0x00020000);
}
__device__ __forceinline__ cg_f2 cg_ld2(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(cg_f2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0));
}
__device__ __forceinline__ cg_f4 cg_ld4(__amdgpu_buffer_rsrc_t r, unsigned voff) {
  return __builtin_bit_cast(cg_f4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, 0));
}
__device__ __forceinline__ void cg_st4(__amdgpu_buffer_rsrc_t r, unsigned voff, cg_f4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) int, v), r, (int)voff,
                                         0, 0);
}
// lane l <- lane l-1 (wave_shr:1) and lane l <- lane l+1 (wave_shl:1); lanes
// without a source read 0 (bound_ctrl)
__device__ __forceinline__ float cg_from_left(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float cg_from_right(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}

struct CgCoef {  // one row, the lane's two pixels (x: first, y: second)
  cg_f2 wxu, wyu, wxv, wyv, a, c, d;
  float wlu, wlv;  // weight of the edge to the left of the first pixel
};

template <bool ODD>
__device__ __forceinline__ cg_f2 cg_mask1(cg_f2 v, bool ok1) {
  if (ODD && !ok1) v.y = 0.f;
  return v;
}
template <bool ODD>
__device__ __forceinline__ cg_f4 cg_mask1(cg_f4 v, bool ok1) {
  if (ODD && !ok1) { v.z = 0.f; v.w = 0.f; }
  return v;
}

// (A f)(row) for f = (u0, v0, u1, v1) rows up / mid / dn; wu = vertical
// weights of the row above (u: .x/.y = pixel 0/1 of wyu, v likewise)
__device__ __forceinline__ cg_f4 cg_apply(cg_f4 up, cg_f4 mid, cg_f4 dn, const CgCoef &c, cg_f2 wuu, cg_f2 wuv) {
  const float Lu = cg_from_left(mid.z), Lv = cg_from_left(mid.w);
  const float Ru = cg_from_right(mid.x), Rv = cg_from_right(mid.y);
  const float s0u = c.wlu * Lu + c.wxu.x * mid.z + wuu.x * up.x + c.wyu.x * dn.x;
  const float s0v = c.wlv * Lv + c.wxv.x * mid.w + wuv.x * up.y + c.wyv.x * dn.y;
  const float s1u = c.wxu.x * mid.x + c.wxu.y * Ru + wuu.y * up.z + c.wyu.y * dn.z;
  const float s1v = c.wxv.x * mid.y + c.wxv.y * Rv + wuv.y * up.w + c.wyv.y * dn.w;
  cg_f4 o;
  o.x = c.a.x * mid.x + c.c.x * mid.y - s0u;
  o.y = c.c.x * mid.x + c.d.x * mid.y - s0v;
  o.z = c.a.y * mid.z + c.c.y * mid.w - s1u;
  o.w = c.c.y * mid.z + c.d.y * mid.w - s1v;
  return o;
}

// inverse of the preconditioner block of both pixels: (ia, ic, id) with
// M^-1 (ru, rv) = (ia ru + ic rv, ic ru + id rv)
struct CgInv {
  cg_f2 ia, ic, id;
};
template <bool BLOCK>
__device__ __forceinline__ CgInv cg_inv(const CgCoef &c) {
  CgInv o;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const float a = c.a[e], cc = c.c[e], d = c.d[e];
    // scalar Jacobi, base.py:129-131: 1/diag where |diag| > 1e-12 else 0
    float ia = fabsf(a) > 1e-12f ? __builtin_amdgcn_rcpf(a) : 0.f;
    float id = fabsf(d) > 1e-12f ? __builtin_amdgcn_rcpf(d) : 0.f;
    float ic = 0.f;
    if (BLOCK) {
      // explicit fma: the same rounding wherever the inverse is formed
      const float det = __builtin_fmaf(a, d, -(cc * cc));
      const bool ok = det > 1e-30f * fabsf(a * d);
      const float inv = __builtin_amdgcn_rcpf(det);
      ia = ok ? d * inv : ia;
      id = ok ? a * inv : id;
      ic = ok ? -cc * inv : 0.f;
    }
    o.ia[e] = ia;
    o.ic[e] = ic;
    o.id[e] = id;
  }
  return o;
}
__device__ __forceinline__ cg_f4 cg_minv(const CgInv &m, cg_f4 r) {
  cg_f4 z;
  z.x = m.ia.x * r.x + m.ic.x * r.y;
  z.y = m.ic.x * r.x + m.id.x * r.y;
  z.z = m.ia.y * r.z + m.ic.y * r.w;
  z.w = m.ic.y * r.z + m.id.y * r.w;
  return z;
}
__device__ __forceinline__ float cg_dot(cg_f4 a, cg_f4 b) { return a.x * b.x + a.y * b.y + (a.z * b.z + a.w * b.w); }

// The lane's fixed-order partial sums of the 5 arrays of a 256-thread block
// (nb <= PCG_MAX_BLOCKS: at most PCG_MAX_BLOCKS / 256 terms per lane), every
// load issued before the first add.  A loop per array (the earlier form)
// waited for each array's loads before issuing the next array's: five memory
// round trips per launch, the first also draining the pipeline rows issued
// ahead of the prologue.  The same terms in the same order: the same sums.
__device__ __forceinline__ void cg_lane_partials(double (&S)[5], const double *__restrict__ part, int nb, int tid) {
  constexpr int MT = PCG_MAX_BLOCKS / 256;
  double t[MT][5];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int b = tid + m * 256, bc = b < nb ? b : 0;
#pragma unroll
    for (int v = 0; v < 5; ++v) t[m][v] = part[(size_t)v * PCG_MAX_BLOCKS + bc];
  }
#pragma unroll
  for (int v = 0; v < 5; ++v) {
    double s = 0.0;
#pragma unroll
    for (int m = 0; m < MT; ++m) s = tid + m * 256 < nb ? s + t[m][v] : s;
    S[v] = s;
  }
}

// Launch prologue of k_cg / k_cgs: fixed-order sum of the previous launch's
// per-block partials (pq, qz, qMq, rz, rr) -> alpha_{k-1}, rho_k (CG
// recurrence), beta_k, scipy's convergence test; the lead block records the
// state.  Returns true when this launch has nothing to do.
template <bool FIRST>
__device__ __forceinline__ bool cg_prologue(const PcgArgs &g, int k, double *lds, float *alpha, float *beta,
                                            bool *xlo_zero = nullptr) {
  __shared__ int s_exit, s_xz;
  __shared__ float s_ab[2];
  const int tid = threadIdx.x + threadIdx.y * 64;
  int st_done = 0, st_updk = 0;
  double st_atol = 0.0, st_rho = 0.0;
  if (tid == 0) {
    st_done = g.st->done;
    st_atol = g.st->atol;
    st_updk = g.st->upd_k;
    if (k >= 2) st_rho = g.st->rho[(k - 1) & 1];  // launch k-1's recurrence value of r.z
  }
  // after a residual replacement (k_cg_update between launches k-1 and k)
  // S[4] is already the replaced residual's r.r: the update wrote it into
  // launch k-1's partials
  double S[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  if (!FIRST) {
    cg_lane_partials(S, g.part_rd, g.nb, tid);
#pragma unroll
    for (int v = 0; v < 5; ++v) S[v] = wave_sum(S[v]);
    if ((tid & 63) == 0)
#pragma unroll
      for (int v = 0; v < 5; ++v) lds[v * 8 + (tid >> 6)] = S[v];
  }
  __syncthreads();
  if (tid == 0) {
    int done = st_done ? -1 : 0;
    float al = 0.f, be = 0.f;
    const bool xz = !FIRST && st_updk == k;
    s_xz = xz;
    if (!FIRST && !done) {
#pragma unroll
      for (int v = 0; v < 5; ++v) S[v] = lds[v * 8] + lds[v * 8 + 1] + lds[v * 8 + 2] + lds[v * 8 + 3];
      const double rn = sqrt(S[4]);
      const double atol = k == 1 ? g.rtol * rn : st_atol;
      if (k == 1 && S[4] == 0.0) done = 3;
      else if (rn < atol || S[4] == 0.0) done = 1;  // exact solution: nothing left to divide
      const double a_ = S[3] / S[0];
      const double rho = S[3] - 2.0 * a_ * S[1] + a_ * a_ * S[2];
      // p.Ap, r.z or the recurrence's next r.z not positive: fp32 rounding
      // at the noise floor (rtol 0 runs past the representable residual; A
      // and M are SPD, so only rounding makes them vanish): stop there
      if (!done && (!(S[0] > 0.0) || !(S[3] > 0.0) || !(rho > 0.0))) done = 1;
      // the r.z the last sweep formed (S[3]) off the recurrence's prediction
      // of it by more than 10 % (they agree to ~1e-6 above the noise floor):
      // conjugacy is lost, restart with beta = 0 (a preconditioned steepest
      // descent step never increases the A-norm error) instead of letting
      // the recurrence drive the iterate away
      const bool drift = k >= 2 && !(fabs(S[3] - st_rho) <= 0.1 * S[3]);
      if (!done && k - 1 >= g.maxiter) done = 2;
      if (blockIdx.x == 0 && blockIdx.y == 0) {
        if (k == 1) { g.st->bnorm = rn; g.st->atol = atol; }
        g.st->iter = k - 1;
        g.st->rr = S[4];
        g.st->rho[k & 1] = rho;
        if (done) g.st->done = done;
        // residual replacement due (k_cg_update): read by update launches only
        if (!done && g.upd_rel > 0.0 && k >= 2 && rn < g.upd_rel * g.st->bnorm && !g.st->upd_due)
          g.st->upd_due = k;
      }
      al = (float)a_;
      be = drift ? 0.f : (float)(rho / S[3]);
    }
    if (FIRST && blockIdx.x == 0 && blockIdx.y == 0) {
      g.st->iter = 0;
      g.st->maxiter = g.maxiter;
    }
    if (g.hflag && blockIdx.x == 0 && blockIdx.y == 0 && done >= 0) {
      if (done > 0) {
        __hip_atomic_store(&g.hflag->iter, k - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&g.hflag->done, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __hip_atomic_store(&g.hflag->k, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    s_exit = done;
    s_ab[0] = al;
    s_ab[1] = be;
  }
  __syncthreads();
  *alpha = s_ab[0];
  *beta = s_ab[1];
  if (xlo_zero) *xlo_zero = s_xz;
  return s_exit != 0;
}

template <bool FIRST, bool BLOCK, bool ODD>
__global__ __launch_bounds__(256) void k_cg(PcgArgs g, int k, int R, int nbands) {
  __shared__ double lds[64];
  const int H = g.H, W = g.W;
  const unsigned rowb4 = (unsigned)g.P * 4u, rowb8 = (unsigned)g.P * 8u;
  const size_t vbytes = (size_t)H * g.P * 8;
  const __amdgpu_buffer_rsrc_t rc = cg_rsrc(g.coef, g.ps * 7 * 4);
  const __amdgpu_buffer_rsrc_t rin = cg_rsrc(FIRST ? g.b : g.r_in, vbytes);
  const __amdgpu_buffer_rsrc_t rpo = cg_rsrc(g.p_old, vbytes);
  const __amdgpu_buffer_rsrc_t rx = cg_rsrc(g.x, vbytes);
  const __amdgpu_buffer_rsrc_t rro = cg_rsrc(g.r_out, vbytes);
  const __amdgpu_buffer_rsrc_t rpn = cg_rsrc(g.p_new, vbytes);
  const unsigned ps4 = (unsigned)(g.ps * 4);
  // XCD-aware tile order (common.h): neighbouring strips / band groups share
  // their halo rows in one L2.  The partials slot is the tile, so the
  // fixed-order sums (and the iterates) do not depend on the order
  const int tile = of_xcd_tile(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
  const int tby = tile / (int)gridDim.x, tbx = tile - tby * (int)gridDim.x;
  // threadIdx.y is wave-uniform (64 x 4 blocks): make every row index scalar
  const int lane = threadIdx.x, band = tby * 4 + __builtin_amdgcn_readfirstlane(threadIdx.y);
  const int jc = tbx * PCG_SW - 2 + 2 * lane;
  const bool ok0 = jc >= 0 && jc < W, ok1 = jc + 1 < W && jc >= 0;
  const bool out_lane = lane >= 1 && lane <= 62;
  const unsigned off4 = ok0 ? (unsigned)jc * 4u : CG_OOB, off8 = ok0 ? (unsigned)jc * 8u : CG_OOB;
  const unsigned soff8 = ok0 && out_lane ? (unsigned)jc * 8u : CG_OOB;
  const bool live = band < nbands;
  const int r0 = band * R, r1 = min(r0 + R, H);

  auto o4 = [&](int t) { return (unsigned)t < (unsigned)H ? off4 + (unsigned)t * rowb4 : CG_OOB; };
  auto o8 = [&](int t) { return (unsigned)t < (unsigned)H ? off8 + (unsigned)t * rowb8 : CG_OOB; };
  auto load_coef = [&](int t, CgCoef &c) {
    const unsigned v = o4(t);
    c.wxu = cg_mask1<ODD>(cg_ld2(rc, v, 0), ok1);
    c.wyu = cg_mask1<ODD>(cg_ld2(rc, v, ps4), ok1);
    c.wxv = cg_mask1<ODD>(cg_ld2(rc, v, 2 * ps4), ok1);
    c.wyv = cg_mask1<ODD>(cg_ld2(rc, v, 3 * ps4), ok1);
    c.a = cg_mask1<ODD>(cg_ld2(rc, v, 4 * ps4), ok1);
    c.c = cg_mask1<ODD>(cg_ld2(rc, v, 5 * ps4), ok1);
    c.d = cg_mask1<ODD>(cg_ld2(rc, v, 6 * ps4), ok1);
  };
  auto load_wy = [&](int t, cg_f2 &wu, cg_f2 &wv) {
    const unsigned v = o4(t);
    wu = cg_mask1<ODD>(cg_ld2(rc, v, ps4), ok1);
    wv = cg_mask1<ODD>(cg_ld2(rc, v, 3 * ps4), ok1);
  };
  auto load_po = [&](int t) { return FIRST ? cg_f4{0.f, 0.f, 0.f, 0.f} : cg_mask1<ODD>(cg_ld4(rpo, o8(t)), ok1); };
  auto load_rin = [&](int t) { return cg_mask1<ODD>(cg_ld4(rin, o8(t)), ok1); };

  // ---- pipeline preamble (independent of alpha/beta: issued before the
  // prologue's reduction so the two memory round trips overlap).  Rows live
  // in 4-slot register rings indexed by (row - (r0 - 1)) & 3, and the row
  // loop is unrolled by 4, so the pipeline advances without register moves.
  CgCoef C[4];   // coefficients, rows t-2 (vertical weights only) .. t+1
  cg_f4 PO[4];   // p_old, rows t-1 .. t+2
  cg_f4 RI[2];   // r_in, rows t, t+1
  if (live) {
    const int t = r0 - 1;
    load_wy(t - 2, C[2].wyu, C[2].wyv);
    load_coef(t - 1, C[3]);
    load_coef(t, C[0]);
    PO[3] = load_po(t - 1);
    PO[0] = load_po(t);
    PO[1] = load_po(t + 1);
    RI[0] = load_rin(t);
  }

  float alpha = 0.f, beta = 0.f;
  if (cg_prologue<FIRST>(g, k, lds, &alpha, &beta)) return;

  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  if (live) {
    const cg_f4 zero4 = {0.f, 0.f, 0.f, 0.f};
    cg_f4 PP[4] = {zero4, zero4, zero4, zero4};  // p, rows t-2 .. t
    cg_f4 RR[2] = {zero4, zero4}, ZZ[2] = {zero4, zero4}, XX[2] = {zero4, zero4};  // rows t-1, t
    CgInv MI[2];
    C[3].wlu = cg_from_left(C[3].wxu.y);
    C[3].wlv = cg_from_left(C[3].wxv.y);
    MI[1] = cg_inv<BLOCK>(C[3]);
    const bool dm0 = out_lane && ok0, dm1 = out_lane && ok1;  // pixels whose dots count
    for (int t0 = r0 - 1; t0 <= r1; t0 += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u;
        if (t > r1) break;
        CgCoef &cm2 = C[(u + 2) & 3], &cm1 = C[(u + 3) & 3], &c0 = C[u & 3], &cp1 = C[(u + 1) & 3];
        // prefetch: coefficients and r_in of row t+1, p_old of row t+2, x of row t
        load_coef(t + 1, cp1);
        RI[(u + 1) & 1] = load_rin(t + 1);
        PO[(u + 2) & 3] = load_po(t + 2);
        XX[u & 1] = (!FIRST && t >= r0 && t < r1) ? cg_mask1<ODD>(cg_ld4(rx, o8(t)), ok1) : zero4;
        // r, z, p of row t
        c0.wlu = cg_from_left(c0.wxu.y);
        c0.wlv = cg_from_left(c0.wxv.y);
        MI[u & 1] = cg_inv<BLOCK>(c0);
        cg_f4 r = RI[u & 1];
        if (!FIRST) r -= alpha * cg_apply(PO[(u + 3) & 3], PO[u & 3], PO[(u + 1) & 3], c0, cm1.wyu, cm1.wyv);
        const cg_f4 z = cg_minv(MI[u & 1], r);
        cg_f4 p = FIRST ? z : z + beta * PO[u & 3];
        const bool rv = (unsigned)t < (unsigned)H;
        if (!(rv && ok0)) { p.x = 0.f; p.y = 0.f; }
        if (!(rv && ok1)) { p.z = 0.f; p.w = 0.f; }
        PP[u & 3] = p;
        RR[u & 1] = r;
        ZZ[u & 1] = z;
        // finish row t-1
        const int o = t - 1;
        if (o >= r0) {
          const cg_f4 pm1 = PP[(u + 3) & 3], rm1 = RR[(u + 1) & 1], zm1 = ZZ[(u + 1) & 1];
          const cg_f4 q = cg_apply(PP[(u + 2) & 3], pm1, p, cm1, cm2.wyu, cm2.wyv);
          const cg_f4 mq = cg_minv(MI[(u + 1) & 1], q);
          const unsigned so = soff8 + (unsigned)o * rowb8;
          cg_st4(rro, so, rm1);
          cg_st4(rpn, so, pm1);
          cg_st4(rx, so, FIRST ? zero4 : XX[(u + 1) & 1] + alpha * PO[(u + 3) & 3]);
          // per-lane fp32 dots over the two pixels (halo lanes / padding masked)
          cg_f4 qm = q, rm = rm1;  // select, not multiply: halo lanes may hold inf/nan
          if (!dm0) { qm.x = 0.f; qm.y = 0.f; rm.x = 0.f; rm.y = 0.f; }
          if (!dm1) { qm.z = 0.f; qm.w = 0.f; rm.z = 0.f; rm.w = 0.f; }
          acc[0] += (double)cg_dot(pm1, qm);
          acc[1] += (double)cg_dot(qm, zm1);
          acc[2] += (double)cg_dot(qm, mq);
          acc[3] += (double)cg_dot(rm, zm1);
          acc[4] += (double)cg_dot(rm, rm1);
        }
      }
    }
  }
  write_partials<5>(acc, g.part_wr, lds, tile);
}

// ---------------------------------------------------------------------------
// The 'backslash' surrogate iteration (k_cgs below): the fused, q-free CG
// iteration with a degree-CG_DEG (5) polynomial preconditioner in the 2x2
// block-Jacobi splitting A = D - N, B = D^-1 N:
//   M^-1 = (c0 + c1 B + ... + c5 B^5) D^-1,
// the Chebyshev polynomial that minimises max |1 - X p(X)| for the spectrum
// of X = D^-1 A = I - B on [a, 2] (a = 0.04, 0.02 for the robust GNC stages;
// host: cheb_poly; 2 bounds the spectrum because D + N is positive
// semidefinite).  p > 0 there, so M is SPD.  (Round 1 used degree 3: 0.54x
// the iterations of a first-order Neumann preconditioner, 0.27x of block
// Jacobi; degree 5 takes 0.69x the iterations of degree 3.)
//
// z = M^-1 r by Horner, one neighbour exchange per stage:
//   y = D^-1 r,  g4 = c4 y + c5 D^-1 N y,  g3 = c3 y + D^-1 N g4, ...,
//   z = c0 y + D^-1 N g1   (and r.z = c0 r.y + y.N g1).
// The rho recurrence needs q.M^-1 q = sum_i c_i T_i with y_q = D^-1 q,
// v1 = D^-1 N y_q, v2 = D^-1 N v1:  T0 = y_q.q, T1 = y_q.N y_q, T2 = v1.N y_q,
// T3 = v1.N v1, T4 = v2.N v1, T5 = v2.N v2 (each edge counted once, by its
// right / lower pixel).
// Seven stencil stages deep, so a strip carries four halo lanes per side
// (PCG_SWP = 112 output columns, lanes 4..59).  Arithmetic is on (u, v)
// pairs of one pixel (packed fp32: v_pk_fma_f32).  Each row's coefficients
// are staged once into an LDS ring of records (per pixel the (u, v) weight
// pairs of the edges right and below and D^-1 as (ia, ic), (ic, id)) that
// every stage reads; D itself is re-formed from D^-1 where a stage needs it.
// halo lanes per side of a k_cgs strip (2 px each).  Everything a launch
// stores (r, p, x) and the dots p.q, q.z, r.z, r.r are exact with 4 (z
// reaches 6 px out); only the T terms of q.M^-1 q at the strip's first and
// last output columns reach 9-10 px (T5 uses v2 of the left neighbour), so
// they see the DPP's zero beyond lane 0.  That moves only the rho
// recurrence's beta: 5 halo lanes (108 output columns) give the same 479 CG
// iterations per 1080p pair and the same pairs/s (profiles/r3ae_*), so 4.
#ifndef CGS_HALO
#define CGS_HALO 4
#endif
#define PCG_SWP (128 - 4 * CGS_HALO)
#define CG_ROW_OOB 0x40000000u

struct CgRec {  // one LDS-ring row: pixel e of the lane, (u, v) pairs
  cg_f2 wx[2], wy[2];  // weights of the edges right of / below the pixel
  cg_f2 ma[2], mb[2];  // D^-1 columns: (ia, ic), (ic, id)
};
struct CgRaw {  // staged global loads of one coefficient row (plane order)
  cg_f2 wxu, wyu, wxv, wyv, a, c, d;
};

__device__ __forceinline__ cg_f2 cg_lo(cg_f4 v) { return cg_f2{v.x, v.y}; }
__device__ __forceinline__ cg_f2 cg_hi(cg_f4 v) { return cg_f2{v.z, v.w}; }
__device__ __forceinline__ cg_f4 cg_cat(cg_f2 a, cg_f2 b) { return cg_f4{a.x, a.y, b.x, b.y}; }
__device__ __forceinline__ cg_f2 cg_left2(cg_f2 v) { return cg_f2{cg_from_left(v.x), cg_from_left(v.y)}; }
__device__ __forceinline__ cg_f2 cg_right2(cg_f2 v) { return cg_f2{cg_from_right(v.x), cg_from_right(v.y)}; }

// N f of the middle row; wu = vertical weight pairs of the row above
__device__ __forceinline__ cg_f4 cgr_nsum(cg_f4 up, cg_f4 mid, cg_f4 dn, const CgRec &c, const cg_f2 (&wu)[2]) {
  const cg_f2 m0 = cg_lo(mid), m1 = cg_hi(mid);
  const cg_f2 L = cg_left2(m1), Rt = cg_right2(m0), wl = cg_left2(c.wx[1]);
  const cg_f2 s0 = wl * L + c.wx[0] * m1 + wu[0] * cg_lo(up) + c.wy[0] * cg_lo(dn);
  const cg_f2 s1 = c.wx[0] * m0 + c.wx[1] * Rt + wu[1] * cg_hi(up) + c.wy[1] * cg_hi(dn);
  return cg_cat(s0, s1);
}
__device__ __forceinline__ cg_f4 cgr_minv(const CgRec &m, cg_f4 r) {
  const cg_f2 z0 = m.ma[0] * r.x + m.mb[0] * r.y;
  const cg_f2 z1 = m.ma[1] * r.z + m.mb[1] * r.w;
  return cg_cat(z0, z1);
}
// D f with D re-formed from the stored D^-1 (its 2x2 inverse; scalar-Jacobi
// rows, ic = 0, give diag(1/ia, 1/id); all-zero records give D = 0)
__device__ __forceinline__ cg_f4 cgr_diag(const CgRec &m, cg_f4 f) {
  cg_f2 o[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const float ia = m.ma[e].x, ic = m.ma[e].y, id = m.mb[e].y;
    const float det = ia * id - ic * ic;
    const float inv = det != 0.f ? __builtin_amdgcn_rcpf(det) : 0.f;
    const cg_f2 da = cg_f2{id, -ic} * inv, db = cg_f2{-ic, ia} * inv;
    const float fu = e ? f.z : f.x, fv = e ? f.w : f.y;
    o[e] = da * fu + db * fv;
  }
  return cg_cat(o[0], o[1]);
}
// D f from the raw coefficient row (wave 0 still holds it): no inverse
__device__ __forceinline__ cg_f4 cgr_diag_raw(const CgRaw &c, cg_f4 f) {
  const cg_f2 u = cg_f2{f.x, f.z}, v = cg_f2{f.y, f.w};
  const cg_f2 du = c.a * u + c.c * v, dv = c.c * u + c.d * v;
  return cg_f4{du.x, dv.x, du.y, dv.y};
}

// b - A x at pixel (i, j) in fp64 from the fp32 operator; x + x_hi when xh
__device__ __forceinline__ double2 resid_px(const float *__restrict__ coef, size_t ps, const float2 *__restrict__ b,
                                           const float2 *__restrict__ x, const float2 *__restrict__ xh, int i, int j,
                                           int H, int W, int P) {
  const size_t k = (size_t)i * P + j;
  auto xv = [&](size_t e) {
    const float2 a = x ? x[e] : make_float2(0.f, 0.f);
    if (!xh) return make_double2(a.x, a.y);
    const float2 h = xh[e];
    return make_double2((double)a.x + (double)h.x, (double)a.y + (double)h.y);
  };
  const double2 xc = xv(k);
  const float2 bb = b[k];
  double su = (double)bb.x - ((double)coef[4 * ps + k] * xc.x + (double)coef[5 * ps + k] * xc.y);
  double sv = (double)bb.y - ((double)coef[5 * ps + k] * xc.x + (double)coef[6 * ps + k] * xc.y);
  if (j + 1 < W) {
    const double2 n = xv(k + 1);
    su += (double)coef[k] * n.x;
    sv += (double)coef[2 * ps + k] * n.y;
  }
  if (j > 0) {
    const double2 n = xv(k - 1);
    su += (double)coef[k - 1] * n.x;
    sv += (double)coef[2 * ps + k - 1] * n.y;
  }
  if (i + 1 < H) {
    const double2 n = xv(k + P);
    su += (double)coef[ps + k] * n.x;
    sv += (double)coef[3 * ps + k] * n.y;
  }
  if (i > 0) {
    const double2 n = xv(k - P);
    su += (double)coef[ps + k - P] * n.x;
    sv += (double)coef[3 * ps + k - P] * n.y;
  }
  return make_double2(su, sv);
}

// ---------------------------------------------------------------------------
// k_cg_small: a whole CG solve in ONE workgroup, for levels of at most
// CG_SMALL_PX pixels.  At the coarse pyramid levels a fused k_cgs launch is
// latency-bound (~23 us however few rows: its 7-stage row pipeline is walked
// by one wave per band), and a solve is one launch per iteration; here the
// whole solve is one launch.  Textbook preconditioned CG with the control
// flow of scipy.sparse.linalg.cg (base.py:116-136): x0 = 0, stop when
// ||r|| < rtol ||b|| before an iteration, at most maxiter iterations.
// Preconditioner as in the fused kernels: DEG 3 = k_cgs's Chebyshev
// polynomial in the 2x2 block-Jacobi splitting A = D - N (Horner, three
// neighbour sums), DEG 0 = D^-1 (2x2 blocks if BLOCK, else scipy's scalar
// Jacobi).  Vectors live in global memory (L2-resident at these sizes);
// sweeps are separated by workgroup barriers; reductions are fixed-order fp64.
#define CGS_BX 64
#define CGS_BY 16
#ifndef CG_SMALL_PX
#define CG_SMALL_PX 4096
#endif

struct CgSmallArgs {
  const float *coef;  // 7 planes, plane stride ps
  size_t ps;
  const float2 *b;
  float2 *x, *r, *p, *q, *y, *t;
  int H, W, P;
  double rtol;
  int maxiter;
  float poly[8];
  PcgState *st;
  float2 *xh;      // 'backslash': x_hi of the residual replacement (k_cg_update)
  double upd_rel;  // ... done once at ||r|| < upd_rel ||b|| (0: never)
};

template <bool BLOCK>
__device__ __forceinline__ void cgs_inv(const float *cf, size_t ps, size_t k, float &ia, float &ic, float &id) {
  const float a = cf[4 * ps + k], cc = cf[5 * ps + k], d = cf[6 * ps + k];
  ia = fabsf(a) > 1e-12f ? __builtin_amdgcn_rcpf(a) : 0.f;  // base.py:129-131
  id = fabsf(d) > 1e-12f ? __builtin_amdgcn_rcpf(d) : 0.f;
  ic = 0.f;
  if (BLOCK) {
    const float det = a * d - cc * cc;
    const bool ok = det > 1e-30f * fabsf(a * d);
    const float inv = __builtin_amdgcn_rcpf(det);
    ia = ok ? d * inv : ia;
    id = ok ? a * inv : id;
    ic = ok ? -cc * inv : 0.f;
  }
}
template <bool BLOCK>
__device__ __forceinline__ float2 cgs_minv(const float *cf, size_t ps, size_t k, float2 f) {
  float ia, ic, id;
  cgs_inv<BLOCK>(cf, ps, k, ia, ic, id);
  return make_float2(ia * f.x + ic * f.y, ic * f.x + id * f.y);
}
// (N f)(i, j): edge weight x neighbour value over the 4 neighbours, u and v
__device__ __forceinline__ float2 cgs_nsum(const float *cf, size_t ps, const float2 *f, int i, int j, int H, int W,
                                           int P) {
  const size_t k = (size_t)i * P + j;
  float su = 0.f, sv = 0.f;
  if (j > 0) {
    const float2 n = f[k - 1];
    su += cf[k - 1] * n.x;
    sv += cf[2 * ps + k - 1] * n.y;
  }
  if (j + 1 < W) {
    const float2 n = f[k + 1];
    su += cf[k] * n.x;
    sv += cf[2 * ps + k] * n.y;
  }
  if (i > 0) {
    const float2 n = f[k - P];
    su += cf[ps + k - P] * n.x;
    sv += cf[3 * ps + k - P] * n.y;
  }
  if (i + 1 < H) {
    const float2 n = f[k + P];
    su += cf[ps + k] * n.x;
    sv += cf[3 * ps + k] * n.y;
  }
  return make_float2(su, sv);
}
// fixed-order fp64 sum over the workgroup, returned to every thread
__device__ __forceinline__ double cgs_sum(double v, double *lds) {
  const int tid = threadIdx.x + threadIdx.y * CGS_BX;
  v = wave_sum(v);
  if ((tid & 63) == 0) lds[tid >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < CGS_BX * CGS_BY / 64; ++w) s += lds[w];
  __syncthreads();
  return s;
}

#define CGS_FOR_PIXELS(H, W)                                  \
  for (int i = threadIdx.y; i < (H); i += CGS_BY)             \
    for (int j = threadIdx.x; j < (W); j += CGS_BX)

template <int DEG, bool BLOCK>
__global__ __launch_bounds__(CGS_BX *CGS_BY) void k_cg_small(CgSmallArgs g) {
  __shared__ double lds[CGS_BX * CGS_BY / 64];
  const int H = g.H, W = g.W, P = g.P;
  const size_t ps = g.ps;
  const float *cf = g.coef;
  double acc = 0.0;
  CGS_FOR_PIXELS(H, W) {
    const size_t k = (size_t)i * P + j;
    const float2 bb = g.b[k];
    g.x[k] = make_float2(0.f, 0.f);
    g.r[k] = bb;
    g.p[k] = make_float2(0.f, 0.f);
    acc += (double)(bb.x * bb.x + bb.y * bb.y);
  }
  double rr = cgs_sum(acc, lds);
  const double bnorm = sqrt(rr), atol = g.rtol * bnorm;
  double rho_prev = 1.0;
  int it = 0, done = 0, upd = 0;
  for (;; ++it) {
    if (!upd && it > 0 && sqrt(rr) < g.upd_rel * bnorm) {
      // residual replacement (see k_cg_update): r = b - A x in fp64, x_hi = x,
      // x_lo = 0; p and rho_prev are kept
      acc = 0.0;
      CGS_FOR_PIXELS(H, W) {
        const size_t k = (size_t)i * P + j;
        const double2 rv = resid_px(cf, ps, g.b, g.x, nullptr, i, j, H, W, P);
        const float2 rf = make_float2((float)rv.x, (float)rv.y);
        g.r[k] = rf;
        g.xh[k] = g.x[k];
        acc += (double)rf.x * rf.x + (double)rf.y * rf.y;
      }
      rr = cgs_sum(acc, lds);  // (barrier: every x read done)
      CGS_FOR_PIXELS(H, W) g.x[(size_t)i * P + j] = make_float2(0.f, 0.f);
      __syncthreads();
      upd = 1;
    }
    if (rr == 0.0 && it == 0) { done = 3; break; }
    if (sqrt(rr) < atol || rr == 0.0) { done = 1; break; }
    if (it >= g.maxiter) { done = 2; break; }
    // z = M^-1 r (into t), rho = r.z
    acc = 0.0;
    if (DEG == 0) {
      CGS_FOR_PIXELS(H, W) {
        const size_t k = (size_t)i * P + j;
        const float2 rk = g.r[k], z = cgs_minv<BLOCK>(cf, ps, k, rk);
        g.t[k] = z;
        acc += (double)(rk.x * z.x + rk.y * z.y);
      }
    } else {
      // Horner: g_DEG-1 = c_DEG-1 y + c_DEG B y, g_i = c_i y + B g_i+1, z = g_0
      CGS_FOR_PIXELS(H, W) {
        const size_t k = (size_t)i * P + j;
        g.y[k] = cgs_minv<BLOCK>(cf, ps, k, g.r[k]);
      }
      __syncthreads();
      CGS_FOR_PIXELS(H, W) {
        const size_t k = (size_t)i * P + j;
        const float2 ny = cgs_minv<BLOCK>(cf, ps, k, cgs_nsum(cf, ps, g.y, i, j, H, W, P)), yk = g.y[k];
        g.t[k] = make_float2(g.poly[DEG - 1] * yk.x + g.poly[DEG] * ny.x, g.poly[DEG - 1] * yk.y + g.poly[DEG] * ny.y);
      }
      float2 *src = g.t, *dst = g.q;
#pragma unroll
      for (int d = DEG - 2; d >= 0; --d) {
        __syncthreads();
        CGS_FOR_PIXELS(H, W) {
          const size_t k = (size_t)i * P + j;
          const float2 ng = cgs_minv<BLOCK>(cf, ps, k, cgs_nsum(cf, ps, src, i, j, H, W, P)), yk = g.y[k];
          const float2 v = make_float2(g.poly[d] * yk.x + ng.x, g.poly[d] * yk.y + ng.y);
          dst[k] = v;
          if (d == 0) {
            const float2 rk = g.r[k];
            acc += (double)(rk.x * v.x + rk.y * v.y);
          }
        }
        float2 *tmp = src;
        src = dst;
        dst = tmp;
      }
      if (src != g.t) {  // z into t
        __syncthreads();
        CGS_FOR_PIXELS(H, W) {
          const size_t k = (size_t)i * P + j;
          g.t[k] = src[k];
        }
      }
    }
    const double rho = cgs_sum(acc, lds);  // (barrier: t complete)
    const float beta = it == 0 ? 0.f : (float)(rho / rho_prev);
    CGS_FOR_PIXELS(H, W) {
      const size_t k = (size_t)i * P + j;
      const float2 z = g.t[k], pk = g.p[k];
      g.p[k] = make_float2(z.x + beta * pk.x, z.y + beta * pk.y);
    }
    __syncthreads();
    acc = 0.0;
    CGS_FOR_PIXELS(H, W) {  // q = A p = D p - N p
      const size_t k = (size_t)i * P + j;
      const float2 pk = g.p[k], np = cgs_nsum(cf, ps, g.p, i, j, H, W, P);
      const float a = cf[4 * ps + k], cc = cf[5 * ps + k], d = cf[6 * ps + k];
      const float2 qk = make_float2(a * pk.x + cc * pk.y - np.x, cc * pk.x + d * pk.y - np.y);
      g.q[k] = qk;
      acc += (double)(pk.x * qk.x + pk.y * qk.y);
    }
    const double pq = cgs_sum(acc, lds);
    if (!(pq > 0.0) || !(rho > 0.0)) { done = 1; break; }  // underflow (see cg_prologue)
    const float alpha = (float)(rho / pq);
    acc = 0.0;
    CGS_FOR_PIXELS(H, W) {
      const size_t k = (size_t)i * P + j;
      const float2 pk = g.p[k], qk = g.q[k], xk = g.x[k], rk = g.r[k];
      g.x[k] = make_float2(xk.x + alpha * pk.x, xk.y + alpha * pk.y);
      const float2 rn = make_float2(rk.x - alpha * qk.x, rk.y - alpha * qk.y);
      g.r[k] = rn;
      acc += (double)(rn.x * rn.x + rn.y * rn.y);
    }
    rr = cgs_sum(acc, lds);
    rho_prev = rho;
  }
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    g.st->iter = it;
    g.st->done = done;
    g.st->rr = rr;
    g.st->bnorm = bnorm;
    g.st->atol = atol;
    g.st->upd_k = upd;
  }
}
template __global__ void k_cg_small<CG_DEG, true>(CgSmallArgs);
template __global__ void k_cg_small<0, true>(CgSmallArgs);
template __global__ void k_cg_small<0, false>(CgSmallArgs);

// ---------------------------------------------------------------------------
// k_cg_reg: the same whole-solve-in-one-workgroup CG (scipy control flow,
// same preconditioners, the 'backslash' residual replacement) for levels of
// at most CG_REG_PX = 2048 pixels (17x30 and 34x60 at 1080p), with every
// vector in REGISTERS: thread t owns the pixels e = t + 512 m (m < CGR_M) of
// the dense row-major index e = i W + j, holds their coefficients, D^-1 and
// x, r, p, y, g, q, and exchanges neighbour values through a double-buffered
// LDS copy of the one field a stencil application reads (one barrier per
// exchange: 6 per iteration at degree 5), and reduces dot products through
// per-wave LDS slots in a fixed order (one barrier each; deterministic).
// k_cg_small walked every vector through global memory with a barrier per
// sweep: ~14 us per iteration at 17x30 / 34x60.
// 512 threads (2 waves per SIMD: up to 256 VGPRs) x 4 pixels; 1024 x 4
// spilled 656 B/lane at the 128 VGPRs a 1024-thread block allows, 1024 x 2
// still 100 B/lane
#define CGR_T 512
#define CGR_M 4
#define CG_REG_PX (CGR_T * CGR_M)

template <int DEG, bool BLOCK>
__global__ __launch_bounds__(CGR_T) void k_cg_reg(CgSmallArgs g) {
  __shared__ float2 ex[2][CG_REG_PX];
  // (u, v) weights of the edges right of / below every pixel: the left / up
  // weights of pixel e are those of e - 1 / e - W (registers held all four
  // and spilled 100 B/lane at 256 VGPRs)
  __shared__ float2 w_rt[CG_REG_PX], w_dn[CG_REG_PX];
  __shared__ double red[2][CGR_T / 64][2];
  const int tid = threadIdx.x + threadIdx.y * CGS_BX, wv = tid >> 6;
  const int H = g.H, W = g.W, P = g.P, N = H * W;
  const size_t ps = g.ps;
  const float *cf = g.coef;
  int e[CGR_M];
  bool ok[CGR_M], hl[CGR_M], hu[CGR_M];  // pixel owned; has a left / upper neighbour
  // coefficients: weights of the edges right / down (u, v), the 2x2 block
  // (a, c, d) and its inverse (ia, ic, id)
  float wr_u[CGR_M], wd_u[CGR_M], wr_v[CGR_M], wd_v[CGR_M];
  float ca[CGR_M], cc[CGR_M], cd[CGR_M], ia[CGR_M], ic[CGR_M], id[CGR_M];
  float2 x[CGR_M], r[CGR_M], p[CGR_M];
  // pitched offset of owned pixel m (a macro: lambdas taking the arrays by
  // reference made them addressable and spilled them)
#define CGR_KOF(m) ((size_t)((ok[m] ? e[m] : 0) / W) * P + ((ok[m] ? e[m] : 0) % W))
#pragma unroll
  for (int m = 0; m < CGR_M; ++m) {
    e[m] = tid + CGR_T * m;
    ok[m] = e[m] < N;
    const int ee = ok[m] ? e[m] : 0;
    const int i = ee / W, j = ee - i * W;
    const size_t k = (size_t)i * P + j;
    hl[m] = ok[m] && j > 0;
    hu[m] = ok[m] && i > 0;
    wr_u[m] = ok[m] && j + 1 < W ? cf[k] : 0.f;
    wd_u[m] = ok[m] && i + 1 < H ? cf[ps + k] : 0.f;
    wr_v[m] = ok[m] && j + 1 < W ? cf[2 * ps + k] : 0.f;
    wd_v[m] = ok[m] && i + 1 < H ? cf[3 * ps + k] : 0.f;
    if (ok[m]) {
      w_rt[ee] = make_float2(wr_u[m], wr_v[m]);
      w_dn[ee] = make_float2(wd_u[m], wd_v[m]);
    }
    ca[m] = ok[m] ? cf[4 * ps + k] : 0.f;
    cc[m] = ok[m] ? cf[5 * ps + k] : 0.f;
    cd[m] = ok[m] ? cf[6 * ps + k] : 0.f;
    if (ok[m]) {
      cgs_inv<BLOCK>(cf, ps, k, ia[m], ic[m], id[m]);
    } else {
      ia[m] = ic[m] = id[m] = 0.f;
    }
    x[m] = make_float2(0.f, 0.f);
    r[m] = ok[m] ? g.b[k] : make_float2(0.f, 0.f);
    p[m] = make_float2(0.f, 0.f);
  }
  __syncthreads();  // w_rt / w_dn complete
  int buf = 0, rb = 0;
  // left / up weights of owned pixel m (0 without that neighbour)
#define CGR_WL(m) (hl[m] ? w_rt[e[m] - 1] : make_float2(0.f, 0.f))
#define CGR_WU(m) (hu[m] ? w_dn[e[m] - W] : make_float2(0.f, 0.f))
  // neighbour sum N f of owned pixel m after exch(f)
  // (macro, not a lambda taking the array: an array reference kept the
  // Horner temporaries addressable and spilled them to scratch)
#define CGR_EXCH(f)                                  \
  {                                                   \
    _Pragma("unroll") for (int m = 0; m < CGR_M; ++m) \
      if (ok[m]) ex[buf][e[m]] = (f)[m];              \
    __syncthreads();                                  \
  }
#define nsum(m)                                                                                              \
  ({                                                                                                         \
    const float2 *X_ = ex[buf];                                                                              \
    const int c_ = ok[m] ? e[m] : 0;                                                                         \
    const float2 L_ = X_[max(c_ - 1, 0)], R_ = X_[min(c_ + 1, N - 1)], U_ = X_[max(c_ - W, 0)],              \
                 D_ = X_[min(c_ + W, N - 1)];                                                                \
    const float2 a_ = CGR_WL(m), b_ = CGR_WU(m);                                                             \
    make_float2(a_.x * L_.x + wr_u[m] * R_.x + b_.x * U_.x + wd_u[m] * D_.x,                                 \
                a_.y * L_.y + wr_v[m] * R_.y + b_.y * U_.y + wd_v[m] * D_.y);                                \
  })
#define minv(m, f)                                                                                           \
  ({                                                                                                         \
    const float2 f_ = (f);                                                                                   \
    make_float2(ia[m] * f_.x + ic[m] * f_.y, ic[m] * f_.x + id[m] * f_.y);                                   \
  })
  // fixed-order fp64 sums of two per-thread values over the workgroup
  auto reduce2 = [&](double v0, double v1, double &s0, double &s1) {
    v0 = wave_sum(v0);
    v1 = wave_sum(v1);
    if ((tid & 63) == 0) {
      red[rb][wv][0] = v0;
      red[rb][wv][1] = v1;
    }
    __syncthreads();
    s0 = 0.0;
    s1 = 0.0;
#pragma unroll
    for (int w = 0; w < CGR_T / 64; ++w) {
      s0 += red[rb][w][0];
      s1 += red[rb][w][1];
    }
    rb ^= 1;
  };
  double acc0 = 0.0;
#pragma unroll
  for (int m = 0; m < CGR_M; ++m) acc0 += (double)(r[m].x * r[m].x + r[m].y * r[m].y);
  double rr, dummy;
  reduce2(acc0, 0.0, rr, dummy);
  const double bnorm = sqrt(rr), atol = g.rtol * bnorm;
  double rho_prev = 1.0;
  int it = 0, done = 0, upd = 0;
  for (;; ++it) {
    if (!upd && it > 0 && sqrt(rr) < g.upd_rel * bnorm) {
      // residual replacement (see k_cg_update): r = b - A x in fp64, x_hi = x,
      // x_lo = 0; p and rho_prev are kept
      CGR_EXCH(x);
      acc0 = 0.0;
#pragma unroll
      for (int m = 0; m < CGR_M; ++m) {
        const float2 *X = ex[buf];
        const int c = ok[m] ? e[m] : 0;
        const float2 L = X[max(c - 1, 0)], R = X[min(c + 1, N - 1)], U = X[max(c - W, 0)], D = X[min(c + W, N - 1)];
        const float2 bm = ok[m] ? g.b[CGR_KOF(m)] : make_float2(0.f, 0.f);
        const float2 a = CGR_WL(m), b = CGR_WU(m);
        const double su = (double)bm.x - ((double)ca[m] * x[m].x + (double)cc[m] * x[m].y) +
                          (double)a.x * L.x + (double)wr_u[m] * R.x + (double)b.x * U.x +
                          (double)wd_u[m] * D.x;
        const double sv = (double)bm.y - ((double)cc[m] * x[m].x + (double)cd[m] * x[m].y) +
                          (double)a.y * L.y + (double)wr_v[m] * R.y + (double)b.y * U.y +
                          (double)wd_v[m] * D.y;
        r[m] = ok[m] ? make_float2((float)su, (float)sv) : make_float2(0.f, 0.f);
        acc0 += (double)r[m].x * r[m].x + (double)r[m].y * r[m].y;
        if (ok[m]) g.xh[CGR_KOF(m)] = x[m];  // x_hi (read back by k_cg_finalize)
        x[m] = make_float2(0.f, 0.f);
      }
      buf ^= 1;
      reduce2(acc0, 0.0, rr, dummy);
      upd = 1;
    }
    if (rr == 0.0 && it == 0) { done = 3; break; }
    if (sqrt(rr) < atol || rr == 0.0) { done = 1; break; }
    if (it >= g.maxiter) { done = 2; break; }
    // z = M^-1 r (Horner in B = D^-1 N), rho = r.z
    float2 z[CGR_M];
    if (DEG == 0) {
#pragma unroll
      for (int m = 0; m < CGR_M; ++m) z[m] = minv(m, r[m]);
    } else {
      float2 y[CGR_M];
#pragma unroll
      for (int m = 0; m < CGR_M; ++m) y[m] = minv(m, r[m]);
      CGR_EXCH(y);
#pragma unroll
      for (int m = 0; m < CGR_M; ++m) {
        const float2 ny = minv(m, nsum(m));
        z[m] = make_float2(g.poly[DEG - 1] * y[m].x + g.poly[DEG] * ny.x, g.poly[DEG - 1] * y[m].y + g.poly[DEG] * ny.y);
      }
      buf ^= 1;
#pragma unroll
      for (int d = DEG - 2; d >= 0; --d) {
        CGR_EXCH(z);
#pragma unroll
        for (int m = 0; m < CGR_M; ++m) {
          const float2 ng = minv(m, nsum(m));
          z[m] = make_float2(g.poly[d] * y[m].x + ng.x, g.poly[d] * y[m].y + ng.y);
        }
        buf ^= 1;
      }
    }
    acc0 = 0.0;
#pragma unroll
    for (int m = 0; m < CGR_M; ++m) acc0 += (double)(r[m].x * z[m].x + r[m].y * z[m].y);
    double rho;
    reduce2(acc0, 0.0, rho, dummy);
    const float beta = it == 0 ? 0.f : (float)(rho / rho_prev);
#pragma unroll
    for (int m = 0; m < CGR_M; ++m) p[m] = make_float2(z[m].x + beta * p[m].x, z[m].y + beta * p[m].y);
    // q = A p = D p - N p, pq = p.q
    CGR_EXCH(p);
    float2 q[CGR_M];
    acc0 = 0.0;
#pragma unroll
    for (int m = 0; m < CGR_M; ++m) {
      const float2 np = nsum(m);
      q[m] = make_float2(ca[m] * p[m].x + cc[m] * p[m].y - np.x, cc[m] * p[m].x + cd[m] * p[m].y - np.y);
      acc0 += (double)(p[m].x * q[m].x + p[m].y * q[m].y);
    }
    buf ^= 1;
    double pq;
    reduce2(acc0, 0.0, pq, dummy);
    if (!(pq > 0.0) || !(rho > 0.0)) { done = 1; break; }  // underflow (see cg_prologue)
    const float alpha = (float)(rho / pq);
    acc0 = 0.0;
#pragma unroll
    for (int m = 0; m < CGR_M; ++m) {
      x[m] = make_float2(x[m].x + alpha * p[m].x, x[m].y + alpha * p[m].y);
      r[m] = make_float2(r[m].x - alpha * q[m].x, r[m].y - alpha * q[m].y);
      acc0 += (double)(r[m].x * r[m].x + r[m].y * r[m].y);
    }
    reduce2(acc0, 0.0, rr, dummy);
    rho_prev = rho;
  }
#pragma unroll
  for (int m = 0; m < CGR_M; ++m)
    if (ok[m]) {
      g.x[CGR_KOF(m)] = x[m];
    }
  if (tid == 0) {
    g.st->iter = it;
    g.st->done = done;
    g.st->rr = rr;
    g.st->bnorm = bnorm;
    g.st->atol = atol;
    g.st->upd_k = upd;
  }
#undef CGR_EXCH
#undef nsum
#undef minv
#undef CGR_KOF
#undef CGR_WL
#undef CGR_WU
}
template __global__ void k_cg_reg<CG_DEG, true>(CgSmallArgs);
template __global__ void k_cg_reg<0, false>(CgSmallArgs);

// ---------------------------------------------------------------------------
// k_cgs: the degree-CG_DEG (5) iteration above with its pipeline stages
// split over the 4 waves of a block, which all work on ONE band:
//   wave 0: loads, coefficient records -> LDS ring, A) r, y of row n-1
//   wave 1: Horner B) g4 (row n-3), g3 (n-4), g2 (n-5), g1 (n-6)
//   wave 2: D) z, p, x of row n-8, E) q, y_q of row n-9
//   wave 3: F) v1 and T1, T2 (row n-11), v2 and T3..T5 (row n-12)
// with one block barrier per row step; rows cross waves through small LDS
// rings (y, g1, y_q; records in a 14-row ring), a wave's own rows stay in
// registers.  (Round 1's k_cgp gave each wave its own band and the whole
// pipeline: its record ring allowed one wave per SIMD and 1.6x the rows
// read.)  Here 74 KB of LDS per block allow 2 blocks per CU (R = 39 at
// 1080p) and a step costs only the heaviest wave's share.  Stage lags follow
// from one barrier per step: a stage reads rows of another wave produced at
// earlier steps; the band is walked for n in [r0 - 8, r1 + 11] so that every
// row a required stage reads was produced.
// Rejected variants of this kernel (record split over waves 0 / 3, register
// record rings, raw-D stage E, pair-block splitting, trimmed drain loads)
// are recorded with their measurements in DESIGN.md §3; the commits that
// measured them hold their source.
#define CGS_NREC 14
// CGS_W0REG (default 1): wave 0 keeps the records of rows n-1, n-2 it
// formed in registers instead of reading them back from the LDS ring (4
// ds_read_b128 + 2 ds_read_b64 and their wait per row step of the
// pace-setting wave; 184 -> 202 VGPRs, the same 2 waves / SIMD).  Round-5
// A/B, 2 reps, the same flow bitwise (profiles/r5s_cgs_ab.log): isolated
// 200-iteration 1080p solve 3.87 / 3.87 vs 3.96 / 3.92 ms, timed bench 47.95 /
// 47.94 vs 47.94 / 47.87 pairs/s.  Masking the out-of-band rows instead of
// branching over them (one basic block per row step) was 5 % slower as timed.
// Also measured and removed (round 5, profiles/r5u_cgs_w3rec_ab.log): the
// coefficient loads and records moved from wave 0 to wave 3 (one row ahead,
// a 15-row ring): wave 0 101 -> 89 K working cycles per launch but wave 3
// 56 -> 92 K, a 200-iteration 1080p solve 4.19 vs 3.90 ms, 45.0 vs 47.8
// pairs/s, the same flow bitwise.
#ifndef CGS_W0REG
#define CGS_W0REG 1
#endif
// Waves 1 and 3 run at issue priority 1 (0 otherwise), above the
// other lanes' kernels that share their SIMDs in the timed geometry: 45.65 /
// 45.78 / 45.87 vs 45.34 / 45.45 / 45.57 pairs/s, 3 reps each
// (profiles/r4k_prio_ab.log); the same arithmetic

// Load distance in row steps (each step ends at a block barrier, so a load
// issued at step n is waited for at step n + distance): wave 0's coefficient,
// p_old and r_in rows (CGS_PF), wave 2's p_old and x rows (CGS_PF2).  Ring
// sizes are powers of two dividing the 8-step unroll.
#ifndef CGS_PF
#define CGS_PF 2
#endif
#ifndef CGS_PF2
#define CGS_PF2 1
#endif
#define CGS_POW2(n) ((n) <= 1 ? 1 : (n) <= 2 ? 2 : (n) <= 4 ? 4 : 8)
#define CGS_SGN CGS_POW2(CGS_PF + 2)
#define CGS_RIN CGS_POW2(CGS_PF + 1)
#define CGS_W2N CGS_POW2(CGS_PF2 + 1)
static_assert(CGS_PF >= 1 && CGS_PF + 3 <= 8 && CGS_PF2 >= 1 && CGS_PF2 + 1 <= 8, "k_cgs load distances");

// CGS_PHASE_TIMING (tools/micro builds only): per role, the cycles a wave
// spends working and waiting at the row-step barriers
#ifdef CGS_PHASE_TIMING
__device__ unsigned long long g_cgs_t[4][3];  // [role] {work, wait, waves}
#define CGS_T0 unsigned long long cgs_wait = 0, cgs_t_start = clock64();
#define CGS_BAR_BEGIN const unsigned long long cgs_b0 = clock64();
#define CGS_BAR_END cgs_wait += clock64() - cgs_b0;
#define CGS_T1                                                           \
  if (lane == 0) {                                                       \
    const unsigned long long tot = clock64() - cgs_t_start;              \
    atomicAdd(&g_cgs_t[wid][0], tot - cgs_wait);                         \
    atomicAdd(&g_cgs_t[wid][1], cgs_wait);                               \
    atomicAdd(&g_cgs_t[wid][2], 1ull);                                   \
  }
#else
#define CGS_T0
#define CGS_BAR_BEGIN
#define CGS_BAR_END
#define CGS_T1
#endif

template <bool FIRST, bool ODD>
__global__ __launch_bounds__(256) void k_cgs(PcgArgs g, int k, int R, int nbands) {
  __shared__ double lds[64];
  __shared__ float4 ring[CGS_NREC][4][64];  // [row slot][record quarter][lane]
  __shared__ float4 s_y[8][64], s_g1[4][64], s_yq[4][64];
  const int H = g.H, W = g.W;
  const unsigned rowb4 = (unsigned)g.P * 4u, rowb8 = (unsigned)g.P * 8u;
  const size_t vbytes = (size_t)H * g.P * 8;
  const __amdgpu_buffer_rsrc_t rc = cg_rsrc(g.coef, g.ps * 7 * 4);
  const __amdgpu_buffer_rsrc_t rin = cg_rsrc(FIRST ? g.b : g.r_in, vbytes);
  const __amdgpu_buffer_rsrc_t rpo = cg_rsrc(g.p_old, vbytes);
  const __amdgpu_buffer_rsrc_t rx = cg_rsrc(g.x, vbytes);
  const __amdgpu_buffer_rsrc_t rro = cg_rsrc(g.r_out, vbytes);
  const __amdgpu_buffer_rsrc_t rpn = cg_rsrc(g.p_new, vbytes);
  const unsigned ps4 = (unsigned)(g.ps * 4);
  // XCD-aware tile order: blocks b, b + 8, b + 16 ... share an XCD's L2
  // (MI355X_MICROARCH.md, workgroup dispatch), so give each XCD a contiguous
  // run of row-major tiles; its neighbours' column halos are then read
  // through the same L2 at about the same row step
  const int nt = gridDim.x * gridDim.y, lin = blockIdx.x + blockIdx.y * gridDim.x;
  const int xcd = lin & 7, tile = xcd * (nt >> 3) + min(xcd, nt & 7) + (lin >> 3);
  const int lane = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(threadIdx.y), band = tile / gridDim.x;
  const int tid = lane + wid * 64;
  // pipeline role of this wave (A/B, round 2: pairing the roles of two
  // co-resident blocks differently on the SIMDs, role = wid ^ f(block), was
  // no faster: 51.5-54 vs 52 us per 1080p launch)
  const int role = wid;
  const int jc = (tile - band * gridDim.x) * PCG_SWP - 2 * CGS_HALO + 2 * lane;
  const bool ok0 = jc >= 0 && jc < W, ok1 = jc + 1 < W && jc >= 0;
  const bool out_lane = lane >= CGS_HALO && lane < 64 - CGS_HALO;
  const unsigned off4 = ok0 ? (unsigned)jc * 4u : CG_OOB, off8 = ok0 ? (unsigned)jc * 8u : CG_OOB;
  const unsigned soff8 = ok0 && out_lane ? (unsigned)jc * 8u : CG_OOB;
  const bool live = band < nbands;
  // odd bands walk bottom to top, so each band meets its neighbours' halo
  // rows at the same row step (both at the start or both at the end of the
  // walk) and the second read of those rows is served by the XCD's L2.  The
  // walk runs in virtual rows t (orig row H-1-t when flipped); the lower
  // edge of virtual row t is the upper edge of its orig row, i.e. the wy
  // stored at orig row H-2-t.
  const bool flip = band & 1;
  const int rb0 = band * R, rb1 = min(rb0 + R, H);
  const int r0 = flip ? H - rb1 : rb0, r1 = flip ? H - rb0 : rb1;
  const float c0 = g.poly[0], c1 = g.poly[1], c2 = g.poly[2], c3 = g.poly[3], c4 = g.poly[4], c5 = g.poly[5];
  auto orow = [&](int t) { return (unsigned)(flip ? H - 1 - t : t); };
  auto o4 = [&](int t) { return off4 + ((unsigned)t < (unsigned)H ? orow(t) * rowb4 : CG_ROW_OOB); };
  auto o8 = [&](int t) { return off8 + ((unsigned)t < (unsigned)H ? orow(t) * rowb8 : CG_ROW_OOB); };
  auto o4w = [&](int t) {
    return flip ? off4 + ((unsigned)t < (unsigned)(H - 1) ? (unsigned)(H - 2 - t) * rowb4 : CG_ROW_OOB) : o4(t);
  };
  auto load_raw = [&](int t, CgRaw &c) {
    const unsigned v = o4(t), vw = o4w(t);
    c.wxu = cg_mask1<ODD>(cg_ld2(rc, v, 0), ok1);
    c.wyu = cg_mask1<ODD>(cg_ld2(rc, vw, ps4), ok1);
    c.wxv = cg_mask1<ODD>(cg_ld2(rc, v, 2 * ps4), ok1);
    c.wyv = cg_mask1<ODD>(cg_ld2(rc, vw, 3 * ps4), ok1);
    c.a = cg_mask1<ODD>(cg_ld2(rc, v, 4 * ps4), ok1);
    c.c = cg_mask1<ODD>(cg_ld2(rc, v, 5 * ps4), ok1);
    c.d = cg_mask1<ODD>(cg_ld2(rc, v, 6 * ps4), ok1);
  };
  // records are keyed by absolute row (rows >= r0 - 7 >= -7)
  auto rslot = [](int t) { return (t + 2 * CGS_NREC) % CGS_NREC; };
  auto put_rec = [&](int t, const CgRaw &c) {
    CgCoef cc;
    cc.a = c.a;
    cc.c = c.c;
    cc.d = c.d;
    const CgInv mi = cg_inv<true>(cc);
    float4 *q = &ring[rslot(t)][0][lane];
    q[0] = make_float4(c.wxu.x, c.wxv.x, c.wyu.x, c.wyv.x);
    q[64] = make_float4(c.wxu.y, c.wxv.y, c.wyu.y, c.wyv.y);
    q[128] = make_float4(mi.ia.x, mi.ic.x, mi.ic.x, mi.id.x);
    q[192] = make_float4(mi.ia.y, mi.ic.y, mi.ic.y, mi.id.y);
    CgRec r;  // the record as get_rec reads it back
    r.wx[0] = cg_f2{c.wxu.x, c.wxv.x};
    r.wy[0] = cg_f2{c.wyu.x, c.wyv.x};
    r.wx[1] = cg_f2{c.wxu.y, c.wxv.y};
    r.wy[1] = cg_f2{c.wyu.y, c.wyv.y};
    r.ma[0] = cg_f2{mi.ia.x, mi.ic.x};
    r.mb[0] = cg_f2{mi.ic.x, mi.id.x};
    r.ma[1] = cg_f2{mi.ia.y, mi.ic.y};
    r.mb[1] = cg_f2{mi.ic.y, mi.id.y};
    return r;
  };
  auto get_rec = [&](int t) {
    const float4 *q = &ring[rslot(t)][0][lane];
    const float4 a = q[0], b = q[64], c = q[128], d = q[192];
    CgRec r;
    r.wx[0] = cg_f2{a.x, a.y};
    r.wy[0] = cg_f2{a.z, a.w};
    r.wx[1] = cg_f2{b.x, b.y};
    r.wy[1] = cg_f2{b.z, b.w};
    r.ma[0] = cg_f2{c.x, c.y};
    r.mb[0] = cg_f2{c.z, c.w};
    r.ma[1] = cg_f2{d.x, d.y};
    r.mb[1] = cg_f2{d.z, d.w};
    return r;
  };
  auto get_wy = [&](int t, cg_f2 (&wu)[2]) {  // vertical weight pairs only
    const float2 *q = reinterpret_cast<const float2 *>(&ring[rslot(t)][0][lane]);
    const float2 a = q[1], b = q[129];
    wu[0] = cg_f2{a.x, a.y};
    wu[1] = cg_f2{b.x, b.y};
  };
  auto ld4 = [&](float4 (&rg)[4][64], int t) {
    const float4 v = rg[t & 3][lane];
    return cg_f4{v.x, v.y, v.z, v.w};
  };
  auto st4 = [&](float4 (&rg)[4][64], int t, cg_f4 v) { rg[t & 3][lane] = make_float4(v.x, v.y, v.z, v.w); };
  auto load_po = [&](int t) { return FIRST ? cg_f4{0.f, 0.f, 0.f, 0.f} : cg_mask1<ODD>(cg_ld4(rpo, o8(t)), ok1); };
  auto load_rin = [&](int t) { return cg_mask1<ODD>(cg_ld4(rin, o8(t)), ok1); };
  // x_lo = 0 in the launch after a residual replacement (xz, known after
  // the prologue; the preamble's x rows are then dropped)
  bool xz = false;
  auto load_x = [&](int t) {
    return (!FIRST && !xz && t >= r0 && t < r1) ? cg_mask1<ODD>(cg_ld4(rx, o8(t)), ok1) : cg_f4{0.f, 0.f, 0.f, 0.f};
  };
  const bool dm0 = out_lane && ok0, dm1 = out_lane && ok1;
  auto mdot = [&](cg_f4 a, cg_f4 b) {
    const cg_f2 p = cg_lo(a) * cg_lo(b), q = cg_hi(a) * cg_hi(b);
    return (dm0 ? p.x + p.y : 0.f) + (dm1 ? q.x + q.y : 0.f);
  };
  const cg_f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const int ns = r0 - 8, ne = r1 + 11;

  // zeroed rings: rows above the band that no required stage reads
  {
    float4 *z = &ring[0][0][0];
    for (int e = tid; e < CGS_NREC * 4 * 64; e += 256) z[e] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int e = tid; e < 8 * 64; e += 256) (&s_y[0][0])[e] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int e = tid; e < 4 * 64; e += 256) {
      (&s_g1[0][0])[e] = make_float4(0.f, 0.f, 0.f, 0.f);
      (&s_yq[0][0])[e] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // wave 0: raw rows ns-2 .. ns+PF-1, p_old rows ns-2 .. ns+PF-1, r_in rows
  // ns-1 .. ns+PF-2; wave 2: p_old, x of rows ns-8 .. ns-9+PF2 (register
  // rings indexed by (row - ns) mod ring size)
  CgRaw SG[CGS_SGN], SGp[2];
  cg_f4 PO[8], RI[CGS_RIN], PO2[CGS_W2N], XI[CGS_W2N];
  if (live && role == 0) {
    load_raw(ns - 2, SGp[0]);
    load_raw(ns - 1, SGp[1]);
#pragma unroll
    for (int m = 0; m < CGS_PF; ++m) load_raw(ns + m, SG[m]);
    SG[CGS_SGN - 1] = SGp[1];  // raw row ns-1: stage A's D at the first step
#pragma unroll
    for (int m = -2; m < CGS_PF; ++m) PO[m & 7] = load_po(ns + m);
#pragma unroll
    for (int m = -1; m < CGS_PF - 1; ++m) RI[(m + 16) & (CGS_RIN - 1)] = load_rin(ns + m);
  }
  if (live && role == 2) {
#pragma unroll
    for (int m = -8; m < CGS_PF2 - 8; ++m) {
      PO2[(m + 16) & (CGS_W2N - 1)] = load_po(ns + m);
      XI[(m + 16) & (CGS_W2N - 1)] = load_x(ns + m);
    }
  }
  float alpha = 0.f, beta = 0.f;
  if (cg_prologue<FIRST>(g, k, lds, &alpha, &beta, &xz)) return;
  if (xz)
#pragma unroll
    for (int m = 0; m < CGS_W2N; ++m) XI[m] = zero4;

  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  CgRec QA[2];  // CGS_W0REG: wave 0's records of rows n - 2, n - 1 (by R2)
  // row o inside the band (stores and dot products only there)
  auto inband = [&](int o) { return o >= r0 && o < r1; };
  if (live) {
    if (role == 0) {
      QA[0] = put_rec(ns - 2, SGp[0]);  // ring slots of rows ns - 2, ns - 1 at u = 0
      QA[1] = put_rec(ns - 1, SGp[1]);
    }
    __syncthreads();
    CGS_T0
    // issue priority for the pace-setting roles (loads + stage A, and z / p /
    // q) over the Horner and T waves they share a SIMD with: 52 -> 50 us
    // per 1080p launch (A/B, profiles/r2z_cgs_setprio_ab.log; wave 0
    // alone: 51.3)
    if (role == 0 || role == 2) __builtin_amdgcn_s_setprio(2);
    // the Horner and T waves above other kernels' waves on their SIMD (the
    // timed lanes run a fine solve one block per CU beside other lanes' work)
    else __builtin_amdgcn_s_setprio(1);
    // each wave runs its own role's loop (registers of one role only), one
    // block barrier per row step in every role (same step count)
#define CGS_STEPS(...)                                                    \
  for (int n0 = ns; n0 <= ne; n0 += 8) {                                  \
    _Pragma("unroll") for (int u = 0; u < 8; ++u) {                       \
      const int n = n0 + u;                                               \
      if (n > ne) break;                                                  \
      __VA_ARGS__                                                         \
      CGS_BAR_BEGIN                                                       \
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");              \
      __builtin_amdgcn_s_barrier();                                       \
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");              \
      CGS_BAR_END                                                         \
    }                                                                     \
  }
// register-ring index of row n + d: (u + d) mod ring size
#define R8(d) ((u + (d) + 16) & 7)
#define R4(d) ((u + (d) + 16) & 3)
#define R2(d) ((u + (d) + 16) & 1)
#define RSG(d) ((u + (d) + 16) & (CGS_SGN - 1))
#define RRI(d) ((u + (d) + 16) & (CGS_RIN - 1))
#define RW2(d) ((u + (d) + 16) & (CGS_W2N - 1))
    if (role == 0) {
      CGS_STEPS({
        load_raw(n + CGS_PF, SG[RSG(CGS_PF)]);
        PO[R8(CGS_PF)] = load_po(n + CGS_PF);
        RI[RRI(CGS_PF - 1)] = load_rin(n + CGS_PF - 1);
        // A) row n-1: r = r_in - alpha A p_old, y = D^-1 r
#if CGS_W0REG
        const cg_f2 wu[2] = {QA[R2(-2)].wy[0], QA[R2(-2)].wy[1]};  // before row n takes the slot
        const CgRec q1 = QA[R2(-1)];
        QA[R2(0)] = put_rec(n, SG[RSG(0)]);
#else
        put_rec(n, SG[RSG(0)]);
        const CgRec q1 = get_rec(n - 1);
        cg_f2 wu[2];
        get_wy(n - 2, wu);
#endif
        cg_f4 r = RI[RRI(-1)];
        if (!FIRST) r -= alpha * (cgr_diag_raw(SG[RSG(-1)], PO[R8(-1)]) - cgr_nsum(PO[R8(-2)], PO[R8(-1)], PO[R8(0)], q1, wu));
        const cg_f4 y = cgr_minv(q1, r);
        s_y[(n - 1) & 7][lane] = make_float4(y.x, y.y, y.z, y.w);
        const int o = n - 1;
        if (inband(o)) {
          cg_st4(rro, soff8 + orow(o) * rowb8, r);
          acc[4] += (double)mdot(r, r);
          acc[3] += (double)(c0 * mdot(r, y));
        }
      })
    } else if (role == 1) {
      // Horner, degree 5: g4 = c4 y + c5 B y (row n-3), g3 = c3 y + B g4
      // (n-4), g2 = c2 y + B g3 (n-5), g1 = c1 y + B g2 (n-6) -> LDS
      cg_f4 G4[4] = {zero4, zero4, zero4, zero4}, G3[4] = {zero4, zero4, zero4, zero4};
      cg_f4 G2[4] = {zero4, zero4, zero4, zero4};
      auto yrow = [&](int t) {
        const float4 a = s_y[t & 7][lane];
        return cg_f4{a.x, a.y, a.z, a.w};
      };
#define CGS_REC1(d) get_rec(n + (d))
#define CGS_WY1(d, w) \
  cg_f2 w[2];         \
  get_wy(n + (d), w)
#define CGS_Y1(d) yrow(n + (d))
      CGS_STEPS({
        CGS_WY1(-7, w7);
        {
          const CgRec q = CGS_REC1(-3);
          CGS_WY1(-4, wu);
          const cg_f4 y0 = CGS_Y1(-3);
          const cg_f4 ny = cgr_nsum(CGS_Y1(-4), y0, CGS_Y1(-2), q, wu);
          G4[R4(-3)] = c4 * y0 + c5 * cgr_minv(q, ny);
        }
        {
          const CgRec q = CGS_REC1(-4);
          CGS_WY1(-5, wu);
          const cg_f4 ng = cgr_nsum(G4[R4(-5)], G4[R4(-4)], G4[R4(-3)], q, wu);
          G3[R4(-4)] = c3 * CGS_Y1(-4) + cgr_minv(q, ng);
        }
        {
          const CgRec q = CGS_REC1(-5);
          CGS_WY1(-6, wu);
          const cg_f4 ng = cgr_nsum(G3[R4(-6)], G3[R4(-5)], G3[R4(-4)], q, wu);
          G2[R4(-5)] = c2 * CGS_Y1(-5) + cgr_minv(q, ng);
        }
        {
          const CgRec q = CGS_REC1(-6);
          const cg_f4 ng = cgr_nsum(G2[R4(-7)], G2[R4(-6)], G2[R4(-5)], q, w7);
          st4(s_g1, n - 6, c1 * CGS_Y1(-6) + cgr_minv(q, ng));
        }
      })
#undef CGS_REC1
#undef CGS_WY1
#undef CGS_Y1
    } else if (role == 2) {
      cg_f4 PP[4] = {zero4, zero4, zero4, zero4}, ZZ[2] = {zero4, zero4};
      CGS_STEPS({
        PO2[RW2(CGS_PF2 - 8)] = load_po(n + CGS_PF2 - 8);
        XI[RW2(CGS_PF2 - 8)] = load_x(n + CGS_PF2 - 8);
        // D) row n-8: z = c0 y + D^-1 N g1, p = z + beta p_old, x += alpha p_old
        {
          const CgRec q4 = get_rec(n - 8);
          cg_f2 wu[2];
          get_wy(n - 9, wu);
          const cg_f4 ng = cgr_nsum(ld4(s_g1, n - 9), ld4(s_g1, n - 8), ld4(s_g1, n - 7), q4, wu);
          const float4 b = s_y[(n - 8) & 7][lane];
          const cg_f4 yr = {b.x, b.y, b.z, b.w};
          const cg_f4 z = c0 * yr + cgr_minv(q4, ng);
          cg_f4 p = FIRST ? z : z + beta * PO2[RW2(-8)];
          const int o = n - 8;
          const bool rv = (unsigned)o < (unsigned)H;
          if (!(rv && ok0)) { p.x = 0.f; p.y = 0.f; }
          if (!(rv && ok1)) { p.z = 0.f; p.w = 0.f; }
          PP[R4(-8)] = p;
          ZZ[R2(-8)] = z;
          if (inband(o)) {
            const unsigned so = soff8 + orow(o) * rowb8;
            cg_st4(rpn, so, p);
            cg_st4(rx, so, FIRST ? zero4 : XI[RW2(-8)] + alpha * PO2[RW2(-8)]);
            acc[3] += (double)mdot(yr, ng);
          }
        }
        // E) row n-9: q = A p, y_q = D^-1 q
        {
          const CgRec q5 = get_rec(n - 9);
          cg_f2 wu[2];
          get_wy(n - 10, wu);
          const cg_f4 pm = PP[R4(-9)];
          const cg_f4 q = cgr_diag(q5, pm) -
                          cgr_nsum(PP[R4(-10)], pm, PP[R4(-8)], q5, wu);
          const cg_f4 yq = cgr_minv(q5, q);
          st4(s_yq, n - 9, yq);
          const int o = n - 9;
          if (inband(o)) {
            acc[0] += (double)mdot(pm, q);
            acc[1] += (double)mdot(q, ZZ[R2(-9)]);
            acc[2] += (double)(c0 * mdot(q, yq));
          }
        }
      })
    } else {
      // q.M^-1 q = sum_i c_i T_i with v0 = y_q, v1 = B v0, v2 = B v1:
      // T1 = v0.N v0, T2 = v1.N v0 (row n-11); T3 = v1.N v1, T4 = v2.N v1,
      // T5 = v2.N v2 (row n-12; T5 counts each edge once, by its right /
      // lower pixel)
      cg_f4 V1[4] = {zero4, zero4, zero4, zero4}, V2[2] = {zero4, zero4};
      CGS_STEPS({
        // row n's record: raw since wave 0 stored it at step n - 1; stage A
        // reads it at step n + 1
        {
          const CgRec q6 = get_rec(n - 11);
          cg_f2 wu[2];
          get_wy(n - 12, wu);
          const cg_f4 yq = ld4(s_yq, n - 11);
          const cg_f4 ny = cgr_nsum(ld4(s_yq, n - 12), yq, ld4(s_yq, n - 10), q6, wu);
          const cg_f4 v1 = cgr_minv(q6, ny);
          V1[R4(-11)] = v1;
          const int o = n - 11;
          if (inband(o)) {
            const cg_f4 t = (c1 * yq + c2 * v1) * ny;
            acc[2] += (double)((dm0 ? t.x + t.y : 0.f) + (dm1 ? t.z + t.w : 0.f));
          }
        }
        {
          const CgRec q7 = get_rec(n - 12);
          cg_f2 wy7[2];
          get_wy(n - 13, wy7);
          const cg_f4 v1 = V1[R4(-12)];
          const cg_f4 nv = cgr_nsum(V1[R4(-13)], v1, V1[R4(-11)], q7, wy7);
          const cg_f4 v2 = cgr_minv(q7, nv);
          const cg_f4 vu = V2[R2(-13)];
          V2[R2(-12)] = v2;
          const int o = n - 12;
          if (inband(o)) {
            const cg_f2 w0 = cg_lo(v2), w1 = cg_hi(v2);
            const cg_f2 h0 = cg_left2(q7.wx[1]) * cg_left2(w1) + wy7[0] * cg_lo(vu);
            const cg_f2 h1 = q7.wx[0] * w0 + wy7[1] * cg_hi(vu);
            const cg_f4 t = (c3 * v1 + c4 * v2) * nv + (2.0f * c5) * v2 * cg_cat(h0, h1);
            acc[2] += (double)((dm0 ? t.x + t.y : 0.f) + (dm1 ? t.z + t.w : 0.f));
          }
        }
      })
    }
#undef R8
#undef R4
#undef R2
#undef RSG
#undef RRI
#undef RW2
#undef CGS_STEPS
    CGS_T1
  }
  write_partials<5>(acc, g.part_wr, lds);
}

// after the last enqueued iteration: apply the convergence test to the last
// iterate and record the final state (1 block)
__global__ __launch_bounds__(256) void k_pcg_check(PcgArgs g, int k) {
  __shared__ double lds[64];
  if (g.st->done) return;
  float a, b;
  pcg_prologue(g, k, lds, &a, &b);
  if (threadIdx.x == 0 && threadIdx.y == 0 && !g.st->done) {
    g.st->iter = k - 1;
    g.st->done = 2;
  }
}

// ---------------------------------------------------------------------------
// Residual replacement of the 'backslash' surrogate (reliable update,
// Sleijpen & van der Vorst 1996): the fp32 CG's recursive residual drifts
// from b - A x by ~eps |A| |x| (|A||x| / |b| ~ 145 on Classic+NL robust
// stages, tools/fp32_floor.py), 6x the 1e-6 target at 1080p.  Once the
// recursive residual has fallen below upd_rel ||b|| (sqrt(rtol): 1e-3), ONE
// launch between CG launches k-1 and k replaces it by the true residual
// b - A x_{k-1}, evaluated in fp64 (stored fp32) from the fp32 operator, and
// moves x_{k-1} into x_hi; launch k restarts x_lo from 0 (cg_prologue: xz)
// and takes r.r from the replacement.  The second segment's x_lo is small,
// so its own drift is ~1e-3 of the first's and the recursive residual then
// tracks the true residual of x_hi + x_lo (fp64 sum) to the end; the solve's
// result is fl32(x_hi + x_lo) (k_cg_finalize).  p, the partials and the rho
// recurrence are kept (the replacement moves r by ~1e-5 of ||r||, far inside
// the 10 % restart test).  Enqueued every few launches; it acts at most once
// per solve and otherwise returns after its prologue, so the result does not
// depend on how many were enqueued.  Grid: the solve's nb blocks, each
// writing one r.r partial (fixed pixel set and order: deterministic).
// Reads x (halo), b, 7 coefficient planes; writes r, x_hi: 60 B/px.
__global__ __launch_bounds__(256) void k_cg_update(PcgArgs g, int k) {
  __shared__ double lds[64];
  __shared__ int s_act;
  const int tid = threadIdx.x + threadIdx.y * 64;
  if (tid == 0) {
    // every block decides alike: upd_due was set by an earlier CG launch's
    // prologue (its recursive residual below upd_rel ||b||), and st->upd_k
    // is written only with this k
    const int updk = g.st->upd_k;
    s_act = !g.st->done && k >= 2 && (updk == k || (updk == 0 && g.st->upd_due > 0));
  }
  __syncthreads();
  if (!s_act) return;
  const int bid = blockIdx.x + blockIdx.y * gridDim.x;
  const int H = g.H, W = g.W, P = g.P, n = H * W;
  float2 *r = const_cast<float2 *>(g.r_in);
  double acc[1] = {0.0};
  for (int e = bid * 256 + tid; e < n; e += g.nb * 256) {
    const int i = e / W, j = e - i * W;
    const size_t kk = (size_t)i * P + j;
    const double2 rv = resid_px(g.coef, g.ps, g.b, g.x, nullptr, i, j, H, W, P);
    const float2 rf = make_float2((float)rv.x, (float)rv.y);
    r[kk] = rf;
    g.xh[kk] = g.x[kk];
    acc[0] += (double)rf.x * rf.x + (double)rf.y * rf.y;
  }
  // the replaced r.r into launch k-1's partial slot 4, which launch k's
  // prologue sums (each block writes only its own slot; no block of this
  // launch reads the partials)
  write_partials<1>(acc, const_cast<double *>(g.part_rd) + 4 * PCG_MAX_BLOCKS, lds);
  if (tid == 0 && bid == 0) {
    g.st->upd_k = k;
    if (g.hflag) __hip_atomic_store(&g.hflag->upd, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// x_lo is part of the iterate only if a CG launch after the replacement ran
// its sweep: a solve that the replacement itself finished (its residual
// already below atol, declared by launch upd_k, iter = upd_k - 1) never
// restarted x_lo, which then still holds x_hi's copy
__device__ __forceinline__ bool cg_xlo_live(const PcgState *st) { return st->iter >= st->upd_k; }

// the solve's result: x = fl32(x_hi + x_lo) after a residual replacement
// (k_cg_update / k_cg_small), else x unchanged
__global__ __launch_bounds__(256) void k_cg_finalize(float2 *x, const float2 *__restrict__ xh,
                                                     const PcgState *st, int H, int W, int P) {
  if (!st->upd_k) return;
  const bool lo = cg_xlo_live(st);
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    const float2 a = lo ? x[k] : make_float2(0.f, 0.f), h = xh[k];
    x[k] = make_float2((float)((double)a.x + (double)h.x), (float)((double)a.y + (double)h.y));
  }
}

// ---------------------------------------------------------------------------
// Lexicographic SOR, exactly the reference's sweep order (base.py:138-172).
// The reference walks the 2N rows of the CSR matrix in order: all u unknowns
// in Fortran order (index i + j*H: down each column, columns left to right),
// then all v unknowns in the same order, each row relaxed in place
//   x_r <- (1 - w) x_r + w (b_r - sum_{c != r} A_rc x_c) / A_rr
// (rows with |A_rr| < 1e-15 skipped), and stops after the first sweep with
// ||x - x_old|| < tol ||x|| (at most max_iters sweeps, x0 = 0).
//
// With A = D - N (2x2 blocks D = [[a, c], [c, d]], N = edge weights), row
// (i, j) of the u half reads u(i-1, j), u(i, j-1) already relaxed this
// sweep, u(i+1, j), u(i, j+1) not yet, and v(i, j) of the previous sweep;
// the v half reads v neighbours the same way and the NEW u(i, j).  So a
// sweep is a Gauss-Seidel pass over the u plane followed by one over the v
// plane, and the update of (i, j) depends only on (i-1, j) and (i, j-1):
// every anti-diagonal i + j = const may be relaxed at once without changing
// a single operand.  The GPU form keeps the reference's iterate exactly
// (up to fp32 rounding):
//   - a launch is one sweep; each 64-thread block (one wave) owns a strip of
//     64 rows of ONE half (u or v); lane l = row i0 + l walks its own row,
//     and at step t relaxes column t - l, so the wave's active points form an
//     anti-diagonal: the up neighbour (relaxed by lane l-1 at step t-1) and
//     the down neighbour (lane l+1's not-yet-relaxed next point) arrive by
//     DPP lane shifts, left / right are the lane's own previous / next point;
//   - strips hand rows to each other through global memory: strip s needs
//     the relaxed last row of strip s-1 (same half), and the v strip s needs
//     the relaxed u of its own rows; producers publish their completed step
//     count every SOR_G steps (sc1 stores of x, s_waitcnt vmcnt(0), sc1 flag
//     store) and consumers poll with sc1 loads and read x only with sc1 loads
//     (MI355X_MICROARCH.md, hand-off table row 1: no L1 copy of x is ever
//     used, so no acquire fence is needed);
//   - blocks take their strip from a ticket counter in dependency order (u
//     strips 0.., then v strips 0..), so a block only ever waits for blocks
//     that hold lower tickets and are therefore already running: the launch
//     cannot deadlock whatever the dispatch order or occupancy;
//   - the stopping test of sweep k-1 runs in the prologue of launch k on the
//     per-strip fp64 partials (fixed order, so every block agrees), ping-
//     ponged by sweep parity.
// prefetch distance in steps (<= 7: ring of 8) and steps between progress
// publications: 7 / 32 vs 4 / 64 = 0.94 vs 1.15 ms per 480x640 sweep, the
// same iterate (profiles/r3i_sor_ab.log; 16 / 8 steps: 0.89 / 0.91 ms).
// Round 4: 8 steps (the round-3 note that 8 steps changed the iterate was the
// compiler contracting the relaxation differently in that build; with
// sor_relax's explicit fmas every setting gives the same iterate), which lets
// the pipelined kernel's sweeps trail each other closely (driver.hip
// OF_SOR_PIPE_WAVES note).
#ifndef SOR_D
#define SOR_D 7
#endif
#ifndef SOR_G
#define SOR_G 8
#endif
#define SOR_MAXS (PCG_MAX_BLOCKS / 2)

struct SorArgs {
  const float *coef;  // 7 planes {wx_u, wy_u, wx_v, wy_v, a, c, d}, plane stride ps
  const float2 *b;
  float2 *x;
  int H, W, P;
  size_t ps;
  int nstrips;          // strips per half; blocks per launch = 2 * nstrips
  int stride;           // progress stamp of launch k = k * stride + steps done
  unsigned *ticket;     // reset per solve
  int *prog;            // [2][SOR_MAXS] progress stamps, reset per solve
  int *fail;            // set when a hand-off wait gave up (reset per solve)
  const double *part_rd;  // [2 * nstrips][2] (dn, xn) of the previous sweep
  double *part_wr;
  PcgState *st;
  float omega;
  double tol;
  int maxiter;
};

__device__ __forceinline__ float2 sor_ld(const float2 *p) {
  const uint64_t v = __hip_atomic_load((const uint64_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_bit_cast(float2, v);
}
__device__ __forceinline__ void sor_st(float2 *p, float2 v) {
  __hip_atomic_store((uint64_t *)p, __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int sor_poll(const int *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// wave-uniform wait until *p >= need (need is wave-uniform).  Bounded: a
// producer that never arrives (a bug, never the schedule: producers hold
// lower tickets) ends the wait after ~2^21 polls with *fail set, so the
// launch always drains; the host turns *fail into an error.
__device__ __forceinline__ void sor_wait(const int *p, int need, int &known, int *fail) {
  for (int n = 0; known < need; ++n) {
    known = __builtin_amdgcn_readfirstlane(sor_poll(p));
    if (known >= need) break;
    if (n > (1 << 21)) {
      if (threadIdx.x == 0) __hip_atomic_store(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      known = need;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
// lane l <- lane l-1 / lane l+1 across the whole wave (ds_bpermute-free:
// row_shr/row_shl cross 16-lane rows only with wave_shr/wave_shl)
__device__ __forceinline__ float sor_from_up(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float sor_from_down(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}

// The relaxation of one point (base.py:161-163), x <- (1 - w) x + w (b -
// sigma) / a_rr with sigma = sum_{c != r} A_rc x_c = -(N x)_r + c x_other,
// shared by k_sor_lex and k_sor_pipe.  Every multiply-add is an explicit
// fmaf and the fp64 sums explicit fma: left to the compiler, the two kernels
// contracted different subsets of the products (the pipelined one packed
// some into v_pk_mul_f32 + v_add), so their iterates differed in the last
// bit; spelled out, the rounding is fixed by the source.
// SOR_RCP: multiply by 1 / a_rr formed at prefetch time instead of dividing
// on the step's dependency chain (an IEEE division is ~8 dependent
// instructions); rounds differently from the division (<= 1.5 ulp)
#ifndef SOR_RCP
#define SOR_RCP 0
#endif
__device__ __forceinline__ float sor_relax(float bb, float wl, float left, float wr, float right, float wd, float down,
                                           float wu, float up, float cc, float other, float dg, float old, float om,
                                           float om1) {
  float sgm = fmaf(wl, left, bb);
  sgm = fmaf(wr, right, sgm);
  sgm = fmaf(wd, down, sgm);
  sgm = fmaf(wu, up, sgm);
  sgm = fmaf(-cc, other, sgm);
#if SOR_RCP
  // dg holds 1 / a_rr here (0 where |a_rr| < 1e-15: the row is skipped)
  return dg == 0.f ? old : fmaf(om1, old, (om * sgm) * dg);
#else
  return fabsf(dg) < 1e-15f ? old : fmaf(om1, old, (om * sgm) / dg);
#endif
}
// v & (c ? ~0 : 0), opaque to the compiler (see the SOR prefetch rings)
__device__ __forceinline__ float sorw_keep(float v, bool c) {
  float r;
  asm("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(0u - (unsigned)c));
  return r;
}
// global (not generic) float pointers: global_load, counted in vmcnt only
typedef const __attribute__((address_space(1))) float sorw_gf;
// the diagonal as sor_relax takes it
__device__ __forceinline__ float sor_dg(float a) {
#if SOR_RCP
  return fabsf(a) < 1e-15f ? 0.f : 1.0f / a;
#else
  return a;
#endif
}
// ||x_new - x_old||^2 and ||x_new||^2 partial sums (fp64)
__device__ __forceinline__ void sor_acc(float nw, float old, double &dn, double &xn) {
  const double dd = (double)nw - (double)old;
  dn = fma(dd, dd, dn);
  xn = fma((double)nw, (double)nw, xn);
}

// one strip of one half: PH 0 relaxes u (x.x), PH 1 relaxes v (x.y)
template <int PH>
__device__ __forceinline__ void sor_strip(const SorArgs &a, int s, int k, double &dn, double &xn) {
  const int lane = threadIdx.x, H = a.H, W = a.W, P = a.P;
  const int i0 = s * 64, i = i0 + lane;
  const bool rowok = i < H;
  const size_t ps = a.ps;
  const float *wxp = a.coef + (PH ? 2 : 0) * ps, *wyp = a.coef + (PH ? 3 : 1) * ps;
  const float *dgp = a.coef + (PH ? 6 : 4) * ps, *ccp = a.coef + 5 * ps;
  const size_t row = (size_t)(rowok ? i : 0) * P;
  const bool has_up = s > 0, has_dn = i0 + 64 < H;
  const size_t row_up = (size_t)(has_up ? i0 - 1 : 0) * P, row_dn = (size_t)(has_dn ? i0 + 64 : 0) * P;
  const int nsteps = W + 63;
  const int base = k * a.stride;
  int *my = a.prog + PH * SOR_MAXS + s;
  const int *pup = a.prog + PH * SOR_MAXS + (s > 0 ? s - 1 : 0);
  const int *pu = a.prog + s;  // v half: the u strip of the same rows
  int known_up = 0, known_u = 0;
  const float om = a.omega, om1 = 1.0f - a.omega;

  // prefetch ring: column j of lane l lives in slot (j + l) & 7 = t & 7
  float2 X[8], XU[8], XD[8];
  float WX[8], WY[8], DG[8], CC[8], BB[8], WYU[8];
  auto fetch = [&](int t) {  // column t + SOR_D - lane
    const int tp = t + SOR_D, jp = tp - lane, q = tp & 7;
    // wave-uniform waits before reading relaxed values of other strips
    // lane 0 reads row i0-1 at column tp: strip s-1's lane 63 relaxes it at
    // its step tp + 63
    if (has_up && tp >= 0 && tp < W) sor_wait(pup, base + tp + 64, known_up, a.fail);
    // v half: lane l reads the relaxed u of (i0 + l, tp - l), done at the u
    // strip's step tp
    if (PH == 1 && tp >= 0 && tp < nsteps) sor_wait(pu, base + tp + 1, known_u, a.fail);
    const bool ok = rowok && jp >= 0 && jp < W;
    const size_t o = row + (ok ? jp : 0);
    X[q] = ok ? sor_ld(a.x + o) : make_float2(0.f, 0.f);
    WX[q] = ok && jp + 1 < W ? wxp[o] : 0.f;
    WY[q] = ok && i + 1 < H ? wyp[o] : 0.f;
    DG[q] = ok ? sor_dg(dgp[o]) : 0.f;
    CC[q] = ok ? ccp[o] : 0.f;
    BB[q] = ok ? (PH ? a.b[o].y : a.b[o].x) : 0.f;
    if (lane == 0) {
      const bool u = has_up && jp >= 0 && jp < W;
      XU[q] = u ? sor_ld(a.x + row_up + jp) : make_float2(0.f, 0.f);
      WYU[q] = u ? wyp[row_up + jp] : 0.f;
    }
    if (lane == 63) {
      const bool d = has_dn && jp >= 0 && jp < W;
      XD[q] = d ? sor_ld(a.x + row_dn + jp) : make_float2(0.f, 0.f);
    }
  };
#pragma unroll
  for (int t = -SOR_D; t < 0; ++t) fetch(t);

  float res = 0.f, wx_prev = 0.f, wy_prev = 0.f;
  for (int t0 = 0; t0 < nsteps; t0 += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = t0 + u;
      if (t >= nsteps) break;
      fetch(t);
      const int j = t - lane, q = t & 7, q1 = (t + 1) & 7;
      const bool act = rowok && j >= 0 && j < W;
      const float2 xo = X[q];
      const float old = PH ? xo.y : xo.x, other = PH ? xo.x : xo.y;
      // right neighbour: this lane's next point (not yet relaxed)
      const float right = PH ? X[q1].y : X[q1].x;
      // down neighbour: lane l+1's next point; the last lane reads strip s+1
      float down = sor_from_down(right);
      if (lane == 63) down = PH ? XD[q].y : XD[q].x;
      // up neighbour: lane l-1's point of the previous step; lane 0 strip s-1
      float up = sor_from_up(res), wu = sor_from_up(wy_prev);
      if (lane == 0) {
        up = PH ? XU[q].y : XU[q].x;
        wu = WYU[q];
      }
      float nw = sor_relax(BB[q], wx_prev, res, WX[q], right, WY[q], down, wu, up, CC[q], other, DG[q], old, om, om1);
      if (act) {
        const size_t o = row + j;
        sor_st(a.x + o, PH ? make_float2(other, nw) : make_float2(nw, other));
        sor_acc(nw, old, dn, xn);
      } else {
        nw = 0.f;
      }
      res = nw;
      wx_prev = act ? WX[q] : 0.f;
      wy_prev = act ? WY[q] : 0.f;
      if (((t + 1) & (SOR_G - 1)) == 0 || t + 1 == nsteps) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(my, base + t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

__global__ __launch_bounds__(64) void k_sor_lex(SorArgs a, int k) {
  __shared__ int s_exit;
  const int lane = threadIdx.x;
  const int nb = 2 * a.nstrips;
  int tk = 0;
  if (lane == 0) tk = (int)atomicAdd(a.ticket, 1u) - k * nb;
  tk = __builtin_amdgcn_readfirstlane(__shfl(tk, 0, 64));
  if (lane == 0) {
    int done = a.st->done ? -1 : 0;
    if (!done && k > 0) {
      double dn = 0.0, xn = 0.0;
      for (int b = 0; b < nb; ++b) {  // fixed order: identical in every block
        dn += a.part_rd[2 * b];
        xn += a.part_rd[2 * b + 1];
      }
      done = sqrt(dn) < a.tol * sqrt(xn) ? 1 : (k >= a.maxiter ? 2 : 0);
      if (tk == 0) {
        a.st->iter = k;
        a.st->rr = dn;
        a.st->xnorm2 = xn;
        if (done) a.st->done = done;
      }
    }
    s_exit = done;
  }
  __syncthreads();
  if (s_exit) return;
  double dn = 0.0, xn = 0.0;
  const int ph = tk >= a.nstrips ? 1 : 0, s = ph ? tk - a.nstrips : tk;
  if (ph) sor_strip<1>(a, s, k, dn, xn);
  else sor_strip<0>(a, s, k, dn, xn);
  dn = wave_sum(dn);
  xn = wave_sum(xn);
  if (lane == 0) {
    const int slot = ph * a.nstrips + s;  // fixed slot per strip: deterministic sums
    a.part_wr[2 * slot] = dn;
    a.part_wr[2 * slot + 1] = xn;
  }
}

__global__ __launch_bounds__(64) void k_sor_init(SorArgs a) {
  for (int e = threadIdx.x + blockIdx.x * 64; e < a.H * a.P; e += gridDim.x * 64) a.x[e] = make_float2(0.f, 0.f);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.st->iter = 0;
    a.st->maxiter = a.maxiter;
    a.st->done = a.maxiter <= 0 ? 2 : 0;
  }
}

// after the last enqueued sweep k-1: its stopping test (1 wave)
__global__ __launch_bounds__(64) void k_sor_final(SorArgs a, int k) {
  if (threadIdx.x != 0 || a.st->done) return;
  double dn = 0.0, xn = 0.0;
  for (int b = 0; b < 2 * a.nstrips; ++b) {
    dn += a.part_rd[2 * b];
    xn += a.part_rd[2 * b + 1];
  }
  a.st->iter = k;
  a.st->rr = dn;
  a.st->xnorm2 = xn;
  a.st->done = sqrt(dn) < a.tol * sqrt(xn) ? 1 : 2;
}

// ---------------------------------------------------------------------------
// Pipelined lexicographic SOR: many sweeps in flight in ONE persistent launch.
//
// k_sor_lex runs one sweep per launch, so sweep k+1 starts only when the last
// strip of sweep k has ended, and a 480x640 sweep keeps 16 waves busy on a
// 1024-SIMD chip.  But Gauss-Seidel in lexicographic order needs, at point
// (i, j) of sweep k+1, only values sweep k has already produced there: the
// old u, v at (i, j), (i, j+1), (i+1, j), which sweep k wrote when its own
// wavefront passed.  So sweep k+1 can trail sweep k at a fixed distance, and
// so on: sweeps k+1, k+2, ... run side by side, each a wavefront behind the
// previous one.  Every point is still relaxed from exactly the operands of
// the reference's order, so the iterate is bitwise the one of k_sor_lex.
//
// Sweep k writes buffer k mod S of a ring of S (its own "new" values) and
// reads the previous sweep's values from buffer (k-1) mod S (sweep 0 from the
// zero field x).  So x_k survives until sweep k+S, and the stopping test of
// sweep k (which needs all of its strips) may be decided after later sweeps
// have started: the first sweep that passes ||x_k - x_{k-1}|| < tol ||x_k||
// sets *stop = k, later sweeps abandon their work, and k_sor_pipe_final
// copies buffer k mod S into x.  A unit (k, half, strip) that would
// overwrite buffer k mod S first waits for sweep k-S's decision.
//
// Units are taken from a ticket counter in dependency order (sweep, then u
// strips, then v strips), by waves of a persistent grid (one wave per CU, the
// configuration of the sc1 hand-off, MI355X_MICROARCH.md "hand-offs" row 1):
// every wait is on a lower ticket, so the launch cannot deadlock.  A unit
// waits (wave-uniform polls of progress stamps = sweep * stride + steps) for
//   - strip s-1 of its own sweep and half (the relaxed row above),
//   - (v half) the u strip of its own rows in its own sweep,
//   - strip s of sweep k-1's v half (old u, v of its rows: the v strip runs
//     behind the u strip, so this covers both) and strip s+1 of sweep k-1's
//     same half (the old row below).
// The stopping test sums the per-strip fp64 partials in the same fixed order
// as k_sor_lex; the last unit of a sweep to finish (an atomic count) decides.
// Every wait is bounded and also ends when *fail or an earlier *stop is seen,
// so the grid always drains.
#define SOR_RING_MAX 32
struct SorPipeArgs {
  const float *coef;  // 7 planes, plane stride ps
  const float2 *b;
  const float2 *x0;   // zero field: the "previous sweep" of sweep 0
  float2 *ring;       // S buffers of H x P float2, stride bstride
  size_t bstride;
  int H, W, P;
  size_t ps;
  int nstrips, S, stride;
  unsigned *ticket;
  int *fail;
  int *stop;          // first sweep whose test passed / hit maxiter (0x7fffffff until then)
  int *cnt;           // [S] finished units per ring slot (monotone)
  int *dec;           // [S] (sweep + 1) * 4 + done code, once decided
  int *prog;          // [S][2][SOR_MAXS] progress stamps
  double *part;       // [S][2 * SOR_MAXS][2] per-strip (dn, xn)
  double *res;        // [S][2] the decided sweep's (dn, xn)
  float omega;
  double tol;
  int maxiter;
};

__device__ __forceinline__ float sor_ld1(const float *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double sor_ldd(const double *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sor_std(double *p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave-uniform wait until *p >= need; false when the unit must be abandoned
// (a later poll of *stop shows an earlier sweep finished the solve, or *fail)
__device__ __forceinline__ bool sorp_wait(const SorPipeArgs &a, const int *p, int need, int &known, int k) {
  for (int n = 0; known < need; ++n) {
    known = __builtin_amdgcn_readfirstlane(sor_poll(p));
    if (known >= need) break;
    if ((n & 31) == 31) {
      const int st = __builtin_amdgcn_readfirstlane(sor_poll(a.stop));
      const int fl = __builtin_amdgcn_readfirstlane(sor_poll(a.fail));
      if (st < k || fl) return false;
    }
    if (n > (1 << 21)) {
      if (threadIdx.x == 0) __hip_atomic_store(a.fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// unit (k, PH, s): strip s of half PH in sweep k; false if abandoned.  The
// relaxation below is k_sor_lex's, operand for operand.
template <int PH>
__device__ __forceinline__ bool sorp_unit(const SorPipeArgs &a, int k, int s, double &dn, double &xn) {
  const int lane = threadIdx.x, H = a.H, W = a.W, P = a.P;
  const int i0 = s * 64, i = i0 + lane;
  const bool rowok = i < H;
  const size_t ps = a.ps;
  const float *wxp = a.coef + (PH ? 2 : 0) * ps, *wyp = a.coef + (PH ? 3 : 1) * ps;
  const float *dgp = a.coef + (PH ? 6 : 4) * ps, *ccp = a.coef + 5 * ps;
  const size_t row = (size_t)(rowok ? i : 0) * P;
  const bool has_up = s > 0, has_dn = i0 + 64 < H;
  const size_t row_up = (size_t)(has_up ? i0 - 1 : 0) * P, row_dn = (size_t)(has_dn ? i0 + 64 : 0) * P;
  const int nsteps = W + 63;
  const int S = a.S, cur = k % S, prv = (k + S - 1) % S;
  float2 *xc = a.ring + (size_t)cur * a.bstride;
  const float2 *xp = k > 0 ? a.ring + (size_t)prv * a.bstride : a.x0;
  const int base = k * a.stride, pbase = (k - 1) * a.stride;
  int *pk = a.prog + cur * 2 * SOR_MAXS;
  const int *pp = a.prog + prv * 2 * SOR_MAXS;
  int *my = pk + PH * SOR_MAXS + s;
  const int *pup = pk + PH * SOR_MAXS + (s > 0 ? s - 1 : 0);
  const int *pu = pk + s;                                       // (k, u, s)
  const int *pold = pp + SOR_MAXS + s;                          // (k-1, v, s)
  const int *pdn = pp + PH * SOR_MAXS + (has_dn ? s + 1 : s);   // (k-1, PH, s+1)
  int known_up = 0, known_u = 0, known_old = 0, known_dn = 0;
  const float om = a.omega, om1 = 1.0f - a.omega;
  bool alive = true;

  float2 X[8], XU[8], XD[8];
  float WX[8], WY[8], DG[8], CC[8], BB[8], WYU[8];
  auto fetch = [&](int t) {  // column t + SOR_D - lane
    const int tp = t + SOR_D, jp = tp - lane, q = tp & 7;
    if (has_up && tp >= 0 && tp < W) alive = alive && sorp_wait(a, pup, base + tp + 64, known_up, k);
    if (PH == 1 && tp >= 0 && tp < nsteps) alive = alive && sorp_wait(a, pu, base + tp + 1, known_u, k);
    if (k > 0 && tp >= 0 && tp < nsteps) alive = alive && sorp_wait(a, pold, pbase + tp + 1, known_old, k);
    if (k > 0 && has_dn && tp - 63 >= 0 && tp - 63 < W)
      alive = alive && sorp_wait(a, pdn, pbase + tp - 62, known_dn, k);
    const bool ok = rowok && jp >= 0 && jp < W;
    const size_t o = row + (ok ? jp : 0);
    if (PH == 0) X[q] = ok ? sor_ld(xp + o) : make_float2(0.f, 0.f);
    else X[q] = ok ? make_float2(sor_ld1((const float *)(xc + o)), sor_ld1((const float *)(xp + o) + 1))
                   : make_float2(0.f, 0.f);
    WX[q] = ok && jp + 1 < W ? wxp[o] : 0.f;
    WY[q] = ok && i + 1 < H ? wyp[o] : 0.f;
    DG[q] = ok ? sor_dg(dgp[o]) : 0.f;
    CC[q] = ok ? ccp[o] : 0.f;
    BB[q] = ok ? (PH ? a.b[o].y : a.b[o].x) : 0.f;
    if (lane == 0) {
      const bool u = has_up && jp >= 0 && jp < W;
      XU[q] = u ? sor_ld(xc + row_up + jp) : make_float2(0.f, 0.f);
      WYU[q] = u ? wyp[row_up + jp] : 0.f;
    }
    if (lane == 63) {
      const bool d = has_dn && jp >= 0 && jp < W;
      XD[q] = d ? sor_ld(xp + row_dn + jp) : make_float2(0.f, 0.f);
    }
  };
#pragma unroll
  for (int t = -SOR_D; t < 0; ++t) fetch(t);
  if (!alive) return false;

  int stop_seen = 0x7fffffff;
  float res = 0.f, wx_prev = 0.f, wy_prev = 0.f;
  for (int t0 = 0; t0 < nsteps; t0 += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = t0 + u;
      if (t >= nsteps) break;
      fetch(t);
      const int j = t - lane, q = t & 7, q1 = (t + 1) & 7;
      const bool act = rowok && j >= 0 && j < W;
      const float2 xo = X[q];
      const float old = PH ? xo.y : xo.x, other = PH ? xo.x : xo.y;
      const float right = PH ? X[q1].y : X[q1].x;
      float down = sor_from_down(right);
      if (lane == 63) down = PH ? XD[q].y : XD[q].x;
      float up = sor_from_up(res), wu = sor_from_up(wy_prev);
      if (lane == 0) {
        up = PH ? XU[q].y : XU[q].x;
        wu = WYU[q];
      }
      float nw = sor_relax(BB[q], wx_prev, res, WX[q], right, WY[q], down, wu, up, CC[q], other, DG[q], old, om, om1);
      if (act) {
        const size_t o = row + j;
        sor_st(xc + o, PH ? make_float2(other, nw) : make_float2(nw, other));
        sor_acc(nw, old, dn, xn);
      } else {
        nw = 0.f;
      }
      res = nw;
      wx_prev = act ? WX[q] : 0.f;
      wy_prev = act ? WY[q] : 0.f;
      if (((t + 1) & (SOR_G - 1)) == 0 || t + 1 == nsteps) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(my, base + t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // *stop as read at the previous publication (its load had a whole
        // publication interval to return): abandon a sweep past the answer
        if (stop_seen < k || !alive) return false;
        stop_seen = __builtin_amdgcn_readfirstlane(sor_poll(a.stop));
      }
    }
  }
  return alive;
}

__global__ __launch_bounds__(64) void k_sor_pipe(SorPipeArgs a) {
  const int lane = threadIdx.x, n2 = 2 * a.nstrips;
  for (;;) {
    int tk = 0;
    if (lane == 0) tk = (int)atomicAdd(a.ticket, 1u);
    tk = __builtin_amdgcn_readfirstlane(__shfl(tk, 0, 64));
    const int k = tk / n2, r = tk - k * n2;
    if (k >= a.maxiter) return;
    if (__builtin_amdgcn_readfirstlane(sor_poll(a.stop)) < k || __builtin_amdgcn_readfirstlane(sor_poll(a.fail)))
      return;
    const int cur = k % a.S;
    if (k >= a.S) {
      // ring slot `cur` still holds sweep k - S: wait for its decision; if it
      // ended the solve, this and every later unit is void
      int known = 0;
      const int need = (k - a.S + 1) * 4;
      if (!sorp_wait(a, a.dec + cur, need, known, k)) return;
      if (known & 3) return;
    }
    const int ph = r >= a.nstrips ? 1 : 0, s = ph ? r - a.nstrips : r;
    double dn = 0.0, xn = 0.0;
    const bool ok = ph ? sorp_unit<1>(a, k, s, dn, xn) : sorp_unit<0>(a, k, s, dn, xn);
    if (!ok) continue;  // abandoned: the next ticket sees *stop / *fail and ends the wave
    dn = wave_sum(dn);
    xn = wave_sum(xn);
    if (lane == 0) {
      double *pt = a.part + ((size_t)cur * 2 * SOR_MAXS + r) * 2;  // fixed slot per strip, as k_sor_lex
      sor_std(pt, dn);
      sor_std(pt + 1, xn);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int c = atomicAdd(a.cnt + cur, 1) + 1;
      if (c == (k / a.S + 1) * n2) {
        // the last unit of sweep k: its stopping test (k_sor_lex's prologue)
        double sd = 0.0, sx = 0.0;
        for (int b = 0; b < n2; ++b) {
          const double *q = a.part + ((size_t)cur * 2 * SOR_MAXS + b) * 2;
          sd += sor_ldd(q);
          sx += sor_ldd(q + 1);
        }
        const int done = sqrt(sd) < a.tol * sqrt(sx) ? 1 : (k + 1 >= a.maxiter ? 2 : 0);
        sor_std(a.res + 2 * cur, sd);
        sor_std(a.res + 2 * cur + 1, sx);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(a.dec + cur, (k + 1) * 4 + done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done) atomicMin(a.stop, k);
      }
    }
  }
}

// after k_sor_pipe: x <- the decided sweep's buffer; the state as k_sor_final
// records it (iter = sweeps done, rr = ||dx||^2, xnorm2 = ||x||^2)
__global__ __launch_bounds__(256) void k_sor_pipe_final(SorPipeArgs a, float2 *x, PcgState *st) {
  const int K = *a.stop;
  if (K == 0x7fffffff || *a.fail) return;
  const int cur = K % a.S;
  const float2 *src = a.ring + (size_t)cur * a.bstride;
  OF_FOR_PIXELS(a.H, a.W) {
    if (j >= a.W) continue;
    const size_t o = (size_t)i * a.P + j;
    x[o] = src[o];
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && threadIdx.y == 0) {
    st->iter = K + 1;
    st->rr = a.res[2 * cur];
    st->xnorm2 = a.res[2 * cur + 1];
    st->done = a.dec[cur] & 3;
  }
}

// ---------------------------------------------------------------------------
// k_sor_wg: the pipelined lexicographic SOR of a small level (<= 64 rows: one
// strip per half) in ONE workgroup, with the sweep ring and the progress
// stamps in LDS.  Same schedule as k_sor_pipe -- unit (sweep k, half) relaxes
// the anti-diagonals of the strip, sweep k+1 trails sweep k, sweep k writes
// ring slot k mod S and reads slot k-1 mod S, a slot is reused only after the
// decision of the sweep that held it -- and the same relaxation operand for
// operand (sor_relax), so the iterate and the sweep count are k_sor_lex's
// bitwise.  What changes is the hand-off: in k_sor_pipe every unit is a wave
// somewhere on the chip, and a sweep's rows reach the next sweep through L2
// (sc1 stores, a stamp every SOR_G steps after s_waitcnt vmcnt(0), polled with
// sc1 loads): ~1 us per hand-off, so at 30x40 a sweep costs ~27 us for ~70
// relaxation steps.  Here the waves share one CU's LDS: a stamp is a ds_write
// and a poll a ds_read.
//
// Units are static: wave w takes tickets w, w + nw, ... in order (ticket 2k =
// (k, u), 2k + 1 = (k, v)); every wait is on a lower ticket (the u unit of
// its sweep, the v unit of the previous sweep, the decision of sweep k - S),
// and all waves of a workgroup are resident, so the lowest unfinished ticket
// can always proceed: no deadlock.  Waits are bounded (fail) and end on an
// earlier decision (stop), so every wave reaches the final barrier.
// waves per workgroup: 8 (2 per SIMD) keep the unit's prefetch ring and both
// halves' code in registers (a 16-wave build has 128 VGPRs and spills)
#define SORW_MAXW 8
struct SorWgArgs {
  const float *coef;  // 7 planes, plane stride ps
  const float2 *b;
  float2 *x;          // the solution (pitched), written from the decided slot
  int H, W, P;
  size_t ps;
  int S, nw;          // ring depth, waves
  float omega;
  double tol;
  int maxiter;
  PcgState *st;
  int *fail;          // global: set when a wait gave up (the host reruns per sweep)
};
struct SorWgShared {  // LDS after the ring
  int prog[SORW_MAXW + 2][2];  // [slot][half] progress stamps (sweep * stride + steps)
  int dec[SORW_MAXW + 2];      // (sweep + 1) * 4 + done code, once decided
  int cnt[SORW_MAXW + 2];      // finished units per slot (monotone)
  double part[SORW_MAXW + 2][2][2];
  double res[SORW_MAXW + 2][2];
  int stop, fail;
};
// LDS stamps without acquire / release: at workgroup scope those also wait
// for the wave's outstanding global loads (s_waitcnt vmcnt(0)), i.e. for the
// coefficient prefetch SOR_D steps ahead, every step (1.5 us per step
// measured), and so does an inline-asm wait with a memory clobber.  Not
// needed: the LDS executes a CU's DS instructions in order, so a unit's data
// ds_writes land before its later stamp ds_write, and a reader's data
// ds_reads (issued after the stamp value they depend on returned) see them.
// Only the compiler must keep LDS accesses on their side of a stamp access:
// signal fences (no instruction).
__device__ __forceinline__ int sorw_ld(const int *p) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  return v;
}
__device__ __forceinline__ void sorw_st(int *p, int v) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
// wave-uniform wait until *p >= need; false when abandoned (an earlier sweep
// decided, or a wait gave up)
__device__ __forceinline__ bool sorw_wait(SorWgShared &sh, const int *p, int need, int &known, int k) {
  for (int n = 0; known < need; ++n) {
    known = __builtin_amdgcn_readfirstlane(sorw_ld(p));
    if (known >= need) break;
    if ((n & 15) == 15 &&
        (__builtin_amdgcn_readfirstlane(sorw_ld(&sh.stop)) < k || __builtin_amdgcn_readfirstlane(sorw_ld(&sh.fail))))
      return false;
    if (n > (1 << 22)) {
      if ((threadIdx.x & 63) == 0) sorw_st(&sh.fail, 1);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// the dynamic LDS of k_sor_wg: [S][H][W] float2 sweep ring, then
// SorWgShared, addressed from the symbol (LDS instructions, not flat ones:
// a flat access counts in both vmcnt and lgkmcnt, so waiting for it would
// also wait for the global coefficient prefetch)
extern __shared__ double sorw_lds[];
__device__ __forceinline__ float2 *sorw_ring() { return reinterpret_cast<float2 *>(sorw_lds); }
__device__ __forceinline__ SorWgShared &sorw_sh(const SorWgArgs &a) {
  return *reinterpret_cast<SorWgShared *>(sorw_ring() + (size_t)a.S * a.H * a.W);
}

template <int PH>
__device__ __forceinline__ bool sorw_unit(const SorWgArgs &a, int k, int stride, double &dn, double &xn) {
  float2 *ring = sorw_ring();
  SorWgShared &sh = sorw_sh(a);
  const int lane = threadIdx.x & 63, H = a.H, W = a.W;
  const bool rowok = lane < H;
  const size_t ps = a.ps;
  // global (not generic) pointers: global_load, counted in vmcnt only
  typedef const __attribute__((address_space(1))) float gf;
  gf *cf = (gf *)a.coef;
  gf *bp = (gf *)a.b + PH;  // b's component of this half (float2 planes)
  gf *wxp = cf + (PH ? 2 : 0) * ps, *wyp = cf + (PH ? 3 : 1) * ps;
  gf *dgp = cf + (PH ? 6 : 4) * ps, *ccp = cf + 5 * ps;
  const size_t row = (size_t)(rowok ? lane : 0) * a.P;
  const int lrow = (rowok ? lane : 0) * W;
  const int nsteps = W + H - 1;  // lane H - 1 relaxes column W - 1 at step W + H - 2
  const int S = a.S, cur = k % S, prv = (k + S - 1) % S;
  float *xc = reinterpret_cast<float *>(ring + (size_t)cur * H * W);
  const float2 *xp = ring + (size_t)prv * H * W;
  const int base = k * stride, pbase = (k - 1) * stride;
  int *my = &sh.prog[cur][PH];
  const int *pu = &sh.prog[cur][0];    // (k, u)
  const int *pold = &sh.prog[prv][1];  // (k - 1, v)
  int known_u = 0, known_old = 0;
  const float om = a.omega, om1 = 1.0f - a.omega;

  // coefficients of column t + SOR_D - lane, SOR_D steps ahead (global, L2)
  float WX[8], WY[8], DG[8], CC[8], BB[8];
  // every load unconditional at a clamped address, the value selected after
  // it: loads under a branch make the compiler wait for all of them
  // (vmcnt(0)) at every step instead of for the one SOR_D steps old
  // The raw values go into the ring and are masked at the step that uses
  // them (+0 where the reference has no entry), by an AND the compiler cannot
  // see through: a mask or select it can see becomes a masked load, whose
  // value is then waited for at once (vmcnt(0)) instead of SOR_D steps later
  auto keep = [](float v, bool c) {
    float r;
    asm("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(0u - (unsigned)c));
    return r;
  };
  auto fetch = [&](int t) {
    const int tp = t + SOR_D, jp = tp - lane, q = tp & 7;
    const size_t o = row + min(max(jp, 0), W - 1);
    WX[q] = wxp[o];
    WY[q] = wyp[o];
    DG[q] = dgp[o];
    CC[q] = ccp[o];
    BB[q] = bp[2 * o];
  };
  // the old (and, for v, this sweep's u) values of column jn of this lane's row
  auto xval = [&](int jn) {
    const bool ok = rowok && jn >= 0 && jn < W;
    const int e = lrow + min(max(jn, 0), W - 1);
    const float2 o = xp[e];
    const float u = PH ? xc[2 * e] : o.x;
    return make_float2(keep(u, ok && (PH || k > 0)), keep(o.y, ok && k > 0));
  };
#pragma unroll
  for (int t = -SOR_D; t < 0; ++t) fetch(t);
  // The waits of a group of 8 steps at once, before the group (a wait in
  // every step made each step ~650 instructions of control flow): step t
  // reads column t + 1 - lane, relaxed by (k-1, v) and (v half) by (k, u) at
  // their step t + 1, so the group [t0, t0 + 7] needs their progress t0 + 9.
  bool alive = true;
  auto group_wait = [&](int t0) {
    const int need = min(t0 + 9, nsteps);
    if (k > 0) alive = alive && sorw_wait(sh, pold, pbase + need, known_old, k);
    if (PH == 1) alive = alive && sorw_wait(sh, pu, base + need, known_u, k);
  };
  group_wait(0);
  if (!alive) return false;
  float2 Xq = xval(-lane);
  float res = 0.f, wx_prev = 0.f, wy_prev = 0.f;
  // whole groups: the steps past nsteps relax nothing (every lane's column
  // is past W) and store nothing
  for (int t0 = 0; t0 < nsteps; t0 += 8) {
    group_wait(t0);
    if (!alive) return false;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = t0 + u;
      fetch(t);
      const float2 Xn = xval(t + 1 - lane);
      const int j = t - lane, q = t & 7;
      const bool act = rowok && j >= 0 && j < W;
      const float wxq = keep(WX[q], act && j + 1 < W), wyq = keep(WY[q], act && lane + 1 < H);
      const float dgq = keep(sor_dg(DG[q]), act), ccq = keep(CC[q], act), bbq = keep(BB[q], act);
      const float old = PH ? Xq.y : Xq.x, other = PH ? Xq.x : Xq.y;
      const float right = PH ? Xn.y : Xn.x;
      float down = sor_from_down(right);
      float up = sor_from_up(res), wu = sor_from_up(wy_prev);
      if (lane == 0) {  // no strip above
        up = 0.f;
        wu = 0.f;
      }
      float nw = sor_relax(bbq, wx_prev, res, wxq, right, wyq, down, wu, up, ccq, other, dgq, old, om, om1);
      if (act) {
        xc[2 * (lrow + j) + PH] = nw;
        sor_acc(nw, old, dn, xn);
      } else {
        nw = 0.f;
      }
      res = nw;
      wx_prev = wxq;
      wy_prev = wyq;
      Xq = Xn;
    }
    if (lane == 0) sorw_st(my, base + min(t0 + 8, nsteps));
  }
  return alive;
}

__global__ __launch_bounds__(SORW_MAXW * 64) void k_sor_wg(SorWgArgs a) {
  float2 *ring = sorw_ring();
  SorWgShared &sh = sorw_sh(a);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int stride = a.W + a.H + 1;  // > steps of a unit
  if (threadIdx.x < SORW_MAXW + 2) {
    sh.prog[threadIdx.x][0] = sh.prog[threadIdx.x][1] = -1;
    sh.dec[threadIdx.x] = 0;
    sh.cnt[threadIdx.x] = 0;
  }
  if (threadIdx.x == 0) {
    sh.stop = 0x7fffffff;
    sh.fail = 0;
  }
  __syncthreads();
  if (wave < a.nw) {
    for (int tk = wave;; tk += a.nw) {
      const int k = tk >> 1, ph = tk & 1;
      if (k >= a.maxiter) break;
      if (__builtin_amdgcn_readfirstlane(sorw_ld(&sh.stop)) < k || __builtin_amdgcn_readfirstlane(sorw_ld(&sh.fail)))
        break;
      const int cur = k % a.S;
      if (k >= a.S) {
        // slot `cur` still holds sweep k - S: wait for its decision; if it
        // ended the solve, this and every later unit is void
        int known = 0;
        if (!sorw_wait(sh, &sh.dec[cur], (k - a.S + 1) * 4, known, k)) break;
        if (known & 3) break;
      }
      double dn = 0.0, xn = 0.0;
      const bool ok = ph ? sorw_unit<1>(a, k, stride, dn, xn) : sorw_unit<0>(a, k, stride, dn, xn);
      if (!ok) break;
      dn = wave_sum(dn);
      xn = wave_sum(xn);
      if (lane == 0) {
        sh.part[cur][ph][0] = dn;
        sh.part[cur][ph][1] = xn;
        const int c = __hip_atomic_fetch_add(&sh.cnt[cur], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) + 1;
        if (c == (k / a.S + 1) * 2) {
          // the last unit of sweep k: its stopping test, k_sor_lex's order
          double sd = 0.0, sx = 0.0;
          for (int b = 0; b < 2; ++b) {
            sd += sh.part[cur][b][0];
            sx += sh.part[cur][b][1];
          }
          const int done = sqrt(sd) < a.tol * sqrt(sx) ? 1 : (k + 1 >= a.maxiter ? 2 : 0);
          sh.res[cur][0] = sd;
          sh.res[cur][1] = sx;
          if (done) __hip_atomic_fetch_min(&sh.stop, k, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
          sorw_st(&sh.dec[cur], (k + 1) * 4 + done);
        }
      }
    }
  }
  __syncthreads();
  const int K = sh.stop;
  if (sh.fail || K == 0x7fffffff) {
    if (threadIdx.x == 0) __hip_atomic_store(a.fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const int cur = K % a.S;
  const float2 *src = ring + (size_t)cur * a.H * a.W;
  for (int e = threadIdx.x; e < a.H * a.W; e += blockDim.x) {
    const int i = e / a.W, j = e - i * a.W;
    a.x[(size_t)i * a.P + j] = src[e];
  }
  if (threadIdx.x == 0) {
    a.st->iter = K + 1;
    a.st->rr = sh.res[cur][0];
    a.st->xnorm2 = sh.res[cur][1];
    a.st->done = sh.dec[cur] & 3;
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
// sum of squares of clip(x) - d (d may be null; clip to [-1, 1] when limit):
// the reference's display norm ||x - duv|| (classic_nl.py:255-256,
// ba.py:189-190, alt_ba.py:249-250), partials for k_norm2_final
__global__ __launch_bounds__(256) void k_step_norm2_part(const float2 *__restrict__ x, const float2 *__restrict__ d,
                                                         int limit, int H, int W, int P, double *part) {
  __shared__ double lds[32];
  double v[1] = {0.0};
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    float2 a = x[k];
    if (limit) a = make_float2(fminf(fmaxf(a.x, -1.f), 1.f), fminf(fmaxf(a.y, -1.f), 1.f));
    const double u = (double)a.x - (d ? (double)d[k].x : 0.0), w = (double)a.y - (d ? (double)d[k].y : 0.0);
    v[0] += u * u + w * w;
  }
  write_partials<1>(v, part, lds);
}
__global__ __launch_bounds__(256) void k_norm2_final(const double *part, int nb, double *result) {
  __shared__ double lds[32];
  double s[1];
  prologue_sum<1>(s, part, nb, lds);
  if (threadIdx.x == 0 && threadIdx.y == 0) *result = s[0];
}

// ---------------------------------------------------------------------------
// Diagnostic: the TRUE residual of a solve, ||b - A x||^2 and ||b||^2 in
// fp64 (A = D - N from the fp32 coefficient planes), independent of any
// solver recurrence.  Per-block partials, then a one-block finish into
// out[0..1].
// fp64 true residual of x (+ x_hi when st says a residual replacement ran)
__global__ __launch_bounds__(256) void k_resid_part(const float *__restrict__ coef, size_t ps,
                                                    const float2 *__restrict__ b, const float2 *__restrict__ x,
                                                    const float2 *__restrict__ xh, const PcgState *st, int H, int W,
                                                    int P, double *part) {
  __shared__ double lds[64];
  double v[2] = {0.0, 0.0};
  const float2 *xhi = xh && st && st->upd_k ? xh : nullptr;
  const float2 *xlo = xhi && !cg_xlo_live(st) ? nullptr : x;
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    const float2 bb = b[k];
    const double2 r = resid_px(coef, ps, b, xlo, xhi, i, j, H, W, P);
    v[0] += r.x * r.x + r.y * r.y;
    v[1] += (double)bb.x * bb.x + (double)bb.y * bb.y;
  }
  write_partials<2>(v, part, lds);
}
__global__ __launch_bounds__(256) void k_resid_final(const double *part, int nb, double *out) {
  __shared__ double lds[64];
  double s[2];
  prologue_sum<2>(s, part, nb, lds);
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    out[0] = s[0];
    out[1] = s[1];
  }
}
