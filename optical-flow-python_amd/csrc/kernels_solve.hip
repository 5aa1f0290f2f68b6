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

struct PcgArgs {
  const float *coef;  // 7 planes, plane stride ps
  float2 *x;
  const float2 *r_in, *p_old;  // iterate k-1
  float2 *r_out, *p_new;       // iterate k
  const float2 *b;
  int H, W, P;
  size_t ps;
  int nb;  // blocks of this grid (== blocks of every launch of the solve)
  double *part;  // [5][PCG_MAX_BLOCKS] partial sums (layout per kernel pair)
  PcgState *st;
  CgFlag *hflag;  // mapped host memory (may be null)
  double rtol;
  int maxiter;
  float poly[4];  // k_cgp: M^-1 = (poly[0] + poly[1] B + poly[2] B^2 + poly[3] B^3) D^-1
};

// the shared prologue: returns 1 when the solve is finished (state written)
__device__ __forceinline__ int pcg_prologue(const PcgArgs &g, int k, double *lds, float *alpha, float *beta) {
  __shared__ int s_exit;
  __shared__ float s_ab[2];
  double S[5];
  prologue_sum<5>(S, g.part, g.nb, lds);  // of K_{k-1}: pq, qz, qMq, rz, rr
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    const bool lead = blockIdx.x == 0 && blockIdx.y == 0;
    const double rn = sqrt(S[4]);
    const double atol = k == 1 ? g.rtol * rn : g.st->atol;
    int done = 0;
    if (k == 1 && S[4] == 0.0) done = 3;
    else if (rn < atol) done = 1;
    else if (k - 1 >= g.maxiter) done = 2;
    const double al = S[3] / S[0];
    const double rho = S[3] - 2.0 * al * S[1] + al * al * S[2];
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
      const float det = a * d - cc * cc;
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

// Launch prologue of k_cg / k_cgn: fixed-order sum of the previous launch's
// per-block partials (pq, qz, qMq, rz, rr) -> alpha_{k-1}, rho_k (CG
// recurrence), beta_k, scipy's convergence test; the lead block records the
// state.  Returns true when this launch has nothing to do.
template <bool FIRST>
__device__ __forceinline__ bool cg_prologue(const PcgArgs &g, int k, double *lds, float *alpha, float *beta) {
  __shared__ int s_exit;
  __shared__ float s_ab[2];
  const int tid = threadIdx.x + threadIdx.y * 64;
  int st_done = 0;
  double st_atol = 0.0;
  if (tid == 0) {
    st_done = g.st->done;
    st_atol = g.st->atol;
  }
  double S[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  if (!FIRST) {
#pragma unroll
    for (int v = 0; v < 5; ++v) {
      double s = 0.0;
      for (int b = tid; b < g.nb; b += 256) s += g.part[(size_t)v * PCG_MAX_BLOCKS + b];
      S[v] = wave_sum(s);
    }
    if ((tid & 63) == 0)
#pragma unroll
      for (int v = 0; v < 5; ++v) lds[v * 8 + (tid >> 6)] = S[v];
  }
  __syncthreads();
  if (tid == 0) {
    int done = st_done ? -1 : 0;
    float al = 0.f, be = 0.f;
    if (!FIRST && !done) {
#pragma unroll
      for (int v = 0; v < 5; ++v) S[v] = lds[v * 8] + lds[v * 8 + 1] + lds[v * 8 + 2] + lds[v * 8 + 3];
      const double rn = sqrt(S[4]);
      const double atol = k == 1 ? g.rtol * rn : st_atol;
      if (k == 1 && S[4] == 0.0) done = 3;
      else if (rn < atol) done = 1;
      else if (k - 1 >= g.maxiter) done = 2;
      const double a_ = S[3] / S[0];
      const double rho = S[3] - 2.0 * a_ * S[1] + a_ * a_ * S[2];
      if (blockIdx.x == 0 && blockIdx.y == 0) {
        if (k == 1) { g.st->bnorm = rn; g.st->atol = atol; }
        g.st->iter = k - 1;
        g.st->rr = S[4];
        g.st->rho[k & 1] = rho;
        if (done) g.st->done = done;
      }
      al = (float)a_;
      be = (float)(rho / S[3]);
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
  // threadIdx.y is wave-uniform (64 x 4 blocks): make every row index scalar
  const int lane = threadIdx.x, band = blockIdx.y * 4 + __builtin_amdgcn_readfirstlane(threadIdx.y);
  const int jc = blockIdx.x * PCG_SW - 2 + 2 * lane;
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
  write_partials<5>(acc, g.part, lds);
}

// ---------------------------------------------------------------------------
// k_cgn: the same fused, q-free CG iteration with the first-order Neumann
// preconditioner of the 2x2 block-Jacobi splitting A = D - N:
//   M^-1 = D^-1 + D^-1 N D^-1,   z = D^-1 (r + N y),  y = D^-1 r
// (symmetric; positive definite since D + N is a signless graph Laplacian
// plus the PSD data blocks).  On Classic+NL stage-2 systems it halves the
// CG iteration count of block Jacobi (measured: 435 -> 217 on RubberWhale,
// 277 -> 138 on a 540x960 synthetic pair) for one more neighbour exchange.
// The recurrence term q.M^-1 q = q.y_q + 2 sum_edges w y_q,i y_q,j (y_q =
// D^-1 q) is accumulated edge by edge: horizontal edges by their left pixel,
// vertical edges by their lower pixel.
//
// Horizontal dependency depth is 3 columns (q <- p <- z <- y <- r <- A
// p_old), so a strip carries two halo lanes per side: PCG_SWN = 120 output
// columns, lanes 2..61.
//
// Pipeline (step t): A) r, y of row t+1 (needs p_old rows t..t+2);
// B) z, p of row t (y rows t-1..t+1), x of row t; C) q = A p, y_q of row
// t-1 (p rows t-2..t), then stores and dot products when t-1 is an output
// row.  Rows live in 4-slot register rings, the loop is unrolled by 4.
// The band is entered at t = r0 - 4 so that y_q of row r0 - 1 exists.

#define PCG_SWN 120

// sum of the neighbour terms N f of the middle row (no diagonal)
__device__ __forceinline__ cg_f4 cg_nsum(cg_f4 up, cg_f4 mid, cg_f4 dn, const CgCoef &c, cg_f2 wuu, cg_f2 wuv) {
  const float Lu = cg_from_left(mid.z), Lv = cg_from_left(mid.w);
  const float Ru = cg_from_right(mid.x), Rv = cg_from_right(mid.y);
  cg_f4 o;
  o.x = c.wlu * Lu + c.wxu.x * mid.z + wuu.x * up.x + c.wyu.x * dn.x;
  o.y = c.wlv * Lv + c.wxv.x * mid.w + wuv.x * up.y + c.wyv.x * dn.y;
  o.z = c.wxu.x * mid.x + c.wxu.y * Ru + wuu.y * up.z + c.wyu.y * dn.z;
  o.w = c.wxv.x * mid.y + c.wxv.y * Rv + wuv.y * up.w + c.wyv.y * dn.w;
  return o;
}
__device__ __forceinline__ cg_f4 cg_diag(const CgCoef &c, cg_f4 f) {
  cg_f4 o;
  o.x = c.a.x * f.x + c.c.x * f.y;
  o.y = c.c.x * f.x + c.d.x * f.y;
  o.z = c.a.y * f.z + c.c.y * f.w;
  o.w = c.c.y * f.z + c.d.y * f.w;
  return o;
}

template <bool FIRST, bool ODD>
__global__ __launch_bounds__(256) void k_cgn(PcgArgs g, int k, int R, int nbands) {
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
  // threadIdx.y is wave-uniform (64 x 4 blocks): make every row index scalar
  const int lane = threadIdx.x, band = blockIdx.y * 4 + __builtin_amdgcn_readfirstlane(threadIdx.y);
  const int jc = blockIdx.x * PCG_SWN - 4 + 2 * lane;
  const bool ok0 = jc >= 0 && jc < W, ok1 = jc + 1 < W && jc >= 0;
  const bool out_lane = lane >= 2 && lane <= 61;
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
  auto load_po = [&](int t) { return FIRST ? cg_f4{0.f, 0.f, 0.f, 0.f} : cg_mask1<ODD>(cg_ld4(rpo, o8(t)), ok1); };
  auto load_rin = [&](int t) { return cg_mask1<ODD>(cg_ld4(rin, o8(t)), ok1); };
  auto load_x = [&](int t) {
    return (!FIRST && t >= r0 && t < r1) ? cg_mask1<ODD>(cg_ld4(rx, o8(t)), ok1) : cg_f4{0.f, 0.f, 0.f, 0.f};
  };
  const cg_f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const cg_f2 zero2 = {0.f, 0.f};

  // rings: slot of row (t0 + u + d) is (u + d) & 3, t0 = r0 - 4 + 4n
  CgCoef C[4];   // coefficients (+ left weights), rows t-1 .. t+1, t+2 loading
  CgInv MI[4];   // D^-1 of the same rows
  cg_f2 WYU[2], WYV[2];  // vertical weights of row t-2
  cg_f4 PO[4];   // p_old rows t .. t+2, t+3 loading
  cg_f4 RI[2];   // r_in rows t+1, t+2 loading
  cg_f4 XI[2];   // x rows t, t+1 loading
  if (live) {
    const int t = r0 - 4;
    C[0].wxu = C[0].wxv = C[0].a = C[0].c = C[0].d = zero2;
    C[0].wlu = C[0].wlv = 0.f;
    {  // row t: only its vertical weights feed stage A of row t+1
      const unsigned v = o4(t);
      C[0].wyu = cg_mask1<ODD>(cg_ld2(rc, v, ps4), ok1);
      C[0].wyv = cg_mask1<ODD>(cg_ld2(rc, v, 3 * ps4), ok1);
    }
    load_coef(t + 1, C[1]);
    PO[0] = load_po(t);
    PO[1] = load_po(t + 1);
    PO[2] = load_po(t + 2);
    RI[1] = load_rin(t + 1);
    XI[0] = zero4;
  }
  float alpha = 0.f, beta = 0.f;
  if (cg_prologue<FIRST>(g, k, lds, &alpha, &beta)) return;

  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  if (live) {
    cg_f4 RR[4] = {zero4, zero4, zero4, zero4};  // r rows t-1 .. t+1
    cg_f4 YY[4] = {zero4, zero4, zero4, zero4};  // y = D^-1 r, rows t-1 .. t+1
    cg_f4 PP[4] = {zero4, zero4, zero4, zero4};  // p rows t-2 .. t
    cg_f4 ZZ[2] = {zero4, zero4};                // z rows t-1, t
    cg_f4 YQ[2] = {zero4, zero4};                // y_q rows t-2, t-1
    WYU[0] = WYU[1] = WYV[0] = WYV[1] = zero2;
    C[2] = C[0];
    C[3] = C[0];
    MI[0] = MI[2] = MI[3] = cg_inv<true>(C[0]);
    const bool dm0 = out_lane && ok0, dm1 = out_lane && ok1;
    for (int t0 = r0 - 4; t0 <= r1; t0 += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u;
        if (t > r1) break;
        CgCoef &cm1 = C[(u + 3) & 3], &c0 = C[u & 3], &cp1 = C[(u + 1) & 3], &cp2 = C[(u + 2) & 3];
        // keep the vertical weights of row t-2, then prefetch row t+2
        WYU[u & 1] = cp2.wyu;
        WYV[u & 1] = cp2.wyv;
        load_coef(t + 2, cp2);
        RI[u & 1] = load_rin(t + 2);
        PO[(u + 3) & 3] = load_po(t + 3);
        XI[(u + 1) & 1] = load_x(t + 1);
        // A) row t+1: r = r_in - alpha A p_old, y = D^-1 r
        cp1.wlu = cg_from_left(cp1.wxu.y);
        cp1.wlv = cg_from_left(cp1.wxv.y);
        MI[(u + 1) & 3] = cg_inv<true>(cp1);
        cg_f4 r = RI[(u + 1) & 1];
        if (!FIRST)
          r -= alpha * (cg_diag(cp1, PO[(u + 1) & 3]) -
                        cg_nsum(PO[u & 3], PO[(u + 1) & 3], PO[(u + 2) & 3], cp1, c0.wyu, c0.wyv));
        {
          const bool rv = (unsigned)(t + 1) < (unsigned)H;
          if (!(rv && ok0)) { r.x = 0.f; r.y = 0.f; }
          if (!(rv && ok1)) { r.z = 0.f; r.w = 0.f; }
        }
        RR[(u + 1) & 3] = r;
        YY[(u + 1) & 3] = cg_minv(MI[(u + 1) & 3], r);
        // B) row t: z = D^-1 (r + N y), p = z + beta p_old, x += alpha p_old
        const cg_f4 z = cg_minv(MI[u & 3], RR[u & 3] + cg_nsum(YY[(u + 3) & 3], YY[u & 3], YY[(u + 1) & 3], c0,
                                                                cm1.wyu, cm1.wyv));
        cg_f4 p = FIRST ? z : z + beta * PO[u & 3];
        {
          const bool rv = (unsigned)t < (unsigned)H;
          if (!(rv && ok0)) { p.x = 0.f; p.y = 0.f; }
          if (!(rv && ok1)) { p.z = 0.f; p.w = 0.f; }
        }
        PP[u & 3] = p;
        ZZ[u & 1] = z;
        if (t >= r0 && t < r1) cg_st4(rx, soff8 + (unsigned)t * rowb8, FIRST ? zero4 : XI[u & 1] + alpha * PO[u & 3]);
        // C) row t-1: q = A p, y_q = D^-1 q; stores and dots for output rows
        const int o = t - 1;
        const cg_f4 pm1 = PP[(u + 3) & 3];
        const CgCoef &cq = cm1;
        const cg_f4 q = cg_diag(cq, pm1) - cg_nsum(PP[(u + 2) & 3], pm1, p, cq, WYU[u & 1], WYV[u & 1]);
        const cg_f4 yq = cg_minv(MI[(u + 3) & 3], q);
        if (o >= r0 && o < r1) {
          const cg_f4 rm1 = RR[(u + 3) & 3], zm1 = ZZ[(u + 1) & 1], yqu = YQ[(u + 1) & 1];
          const unsigned so = soff8 + (unsigned)o * rowb8;
          cg_st4(rro, so, rm1);
          cg_st4(rpn, so, pm1);
          // edge terms of q.M^-1 q: right edges of the lane's pixels, edges
          // to the row above
          const float yRu = cg_from_right(yq.x), yRv = cg_from_right(yq.y);
          const float e0 = cq.wxu.x * yq.x * yq.z + cq.wxv.x * yq.y * yq.w + WYU[u & 1].x * yqu.x * yq.x +
                           WYV[u & 1].x * yqu.y * yq.y;
          const float e1 = cq.wxu.y * yq.z * yRu + cq.wxv.y * yq.w * yRv + WYU[u & 1].y * yqu.z * yq.z +
                           WYV[u & 1].y * yqu.w * yq.w;
          cg_f4 qm = q, rm = rm1;
          float em = 0.f;
          if (dm0) em += e0;
          else { qm.x = 0.f; qm.y = 0.f; rm.x = 0.f; rm.y = 0.f; }
          if (dm1) em += e1;
          else { qm.z = 0.f; qm.w = 0.f; rm.z = 0.f; rm.w = 0.f; }
          acc[0] += (double)cg_dot(pm1, qm);
          acc[1] += (double)cg_dot(qm, zm1);
          acc[2] += (double)(cg_dot(qm, yq) + 2.0f * em);
          acc[3] += (double)cg_dot(rm, zm1);
          acc[4] += (double)cg_dot(rm, rm1);
        }
        YQ[u & 1] = yq;
      }
    }
  }
  write_partials<5>(acc, g.part, lds);
}

// ---------------------------------------------------------------------------
// k_cgp: the fused, q-free CG iteration with a degree-3 polynomial
// preconditioner in the 2x2 block-Jacobi splitting A = D - N, B = D^-1 N:
//   M^-1 = (c0 + c1 B + c2 B^2 + c3 B^3) D^-1,
// the Chebyshev polynomial that minimises max |1 - X p(X)| for the spectrum
// of X = D^-1 A = I - B on [0.04, 2] (host: cheb_poly; 2 bounds the
// spectrum because D + N is positive semidefinite).  p > 0 there, so M is
// SPD.  Measured on Classic+NL stage-2 systems (RubberWhale, 1e-6 relative
// residual): 0.54x the iterations of the first-order Neumann kernel k_cgn.
//
// z = M^-1 r by Horner, one neighbour exchange per stage:
//   y = D^-1 r,  g2 = c2 y + c3 D^-1 N y,  g1 = c1 y + D^-1 N g2,
//   z = c0 y + D^-1 N g1   (and r.z = c0 r.y + y.N g1).
// The rho recurrence needs q.M^-1 q = sum_i c_i T_i with y_q = D^-1 q,
// v1 = D^-1 N y_q:  T0 = y_q.q, T1 = y_q.N y_q, T2 = v1.N y_q (= v1.D v1),
// T3 = v1.N v1 (each edge counted once, by its right / lower pixel).
//
// Pipeline (step n): A) r, y of row n-1; B) g2 of row n-2; C) g1 of row
// n-3; D) z, p, x of row n-4; E) q, y_q of row n-5; F) v1 and the T terms
// of row n-6.  Seven stencil stages deep, so a strip carries four halo
// lanes per side (PCG_SWP = 112 output columns, lanes 4..59) and a band is
// entered at row r0 - 7 and left at r1 + 5.
// Arithmetic is on (u, v) pairs of one pixel (packed fp32: v_pk_fma_f32).
// Each row's coefficients are staged once into a per-wave LDS ring (8 rows;
// per pixel the (u, v) weight pairs of the edges right and below and D^-1
// as (ia, ic), (ic, id); 32 KB per wave) that every stage reads; D itself
// is re-formed from D^-1 where a stage needs it.  Vectors live in register
// rings indexed by (row - (r0 - 7)); the loop is unrolled by eight so every
// ring index is a compile-time constant.  Global loads run two steps ahead
// (coefficients of row n+3, p_old of row n+2), r_in and x one step.
#define PCG_SWP 112
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

template <bool FIRST, bool ODD>
__global__ __launch_bounds__(256) void k_cgp(PcgArgs g, int k, int R, int nbands) {
  __shared__ double lds[64];
  __shared__ float4 ring[4][8][4][64];  // [wave][row slot][record quarter][lane]
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
  // threadIdx.y is wave-uniform (64 x 4 blocks): make every row index scalar
  const int lane = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(threadIdx.y), band = blockIdx.y * 4 + wid;
  const int jc = blockIdx.x * PCG_SWP - 8 + 2 * lane;
  const bool ok0 = jc >= 0 && jc < W, ok1 = jc + 1 < W && jc >= 0;
  const bool out_lane = lane >= 4 && lane <= 59;
  const unsigned off4 = ok0 ? (unsigned)jc * 4u : CG_OOB, off8 = ok0 ? (unsigned)jc * 8u : CG_OOB;
  const unsigned soff8 = ok0 && out_lane ? (unsigned)jc * 8u : CG_OOB;
  const bool live = band < nbands;
  const int r0 = band * R, r1 = min(r0 + R, H);
  const float c0 = g.poly[0], c1 = g.poly[1], c2 = g.poly[2], c3 = g.poly[3];
  // row part of an offset: wave-uniform (SALU); rows outside [0, H) get
  // CG_ROW_OOB, which keeps every lane's sum out of range without wrapping
  // (lane parts are < 2^24 or CG_OOB; buffers < CG_ROW_OOB bytes, host-checked)
  auto o4 = [&](int t) { return off4 + ((unsigned)t < (unsigned)H ? (unsigned)t * rowb4 : CG_ROW_OOB); };
  auto o8 = [&](int t) { return off8 + ((unsigned)t < (unsigned)H ? (unsigned)t * rowb8 : CG_ROW_OOB); };
  auto load_raw = [&](int t, CgRaw &c) {
    const unsigned v = o4(t);
    c.wxu = cg_mask1<ODD>(cg_ld2(rc, v, 0), ok1);
    c.wyu = cg_mask1<ODD>(cg_ld2(rc, v, ps4), ok1);
    c.wxv = cg_mask1<ODD>(cg_ld2(rc, v, 2 * ps4), ok1);
    c.wyv = cg_mask1<ODD>(cg_ld2(rc, v, 3 * ps4), ok1);
    c.a = cg_mask1<ODD>(cg_ld2(rc, v, 4 * ps4), ok1);
    c.c = cg_mask1<ODD>(cg_ld2(rc, v, 5 * ps4), ok1);
    c.d = cg_mask1<ODD>(cg_ld2(rc, v, 6 * ps4), ok1);
  };
  // raw row -> LDS ring slot (per pixel: wx, wy pairs; D^-1 columns)
  auto put_rec = [&](int slot, const CgRaw &c) {
    CgCoef cc;
    cc.a = c.a;
    cc.c = c.c;
    cc.d = c.d;
    const CgInv mi = cg_inv<true>(cc);
    float4 *q = &ring[wid][slot][0][lane];
    q[0] = make_float4(c.wxu.x, c.wxv.x, c.wyu.x, c.wyv.x);
    q[64] = make_float4(c.wxu.y, c.wxv.y, c.wyu.y, c.wyv.y);
    q[128] = make_float4(mi.ia.x, mi.ic.x, mi.ic.x, mi.id.x);
    q[192] = make_float4(mi.ia.y, mi.ic.y, mi.ic.y, mi.id.y);
  };
  auto get_rec = [&](int slot) {
    const float4 *q = &ring[wid][slot][0][lane];
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
  auto get_wy = [&](int slot, cg_f2 (&wu)[2]) {  // vertical weight pairs only
    const float2 *q = reinterpret_cast<const float2 *>(&ring[wid][slot][0][lane]);
    const float2 a = q[1], b = q[129];
    wu[0] = cg_f2{a.x, a.y};
    wu[1] = cg_f2{b.x, b.y};
  };
  auto load_po = [&](int t) { return FIRST ? cg_f4{0.f, 0.f, 0.f, 0.f} : cg_mask1<ODD>(cg_ld4(rpo, o8(t)), ok1); };
  auto load_rin = [&](int t) { return cg_mask1<ODD>(cg_ld4(rin, o8(t)), ok1); };
  auto load_x = [&](int t) {
    return (!FIRST && t >= r0 && t < r1) ? cg_mask1<ODD>(cg_ld4(rx, o8(t)), ok1) : cg_f4{0.f, 0.f, 0.f, 0.f};
  };
  // dot products of output pixels only (select, not multiply: halo lanes
  // may hold inf/nan)
  const bool dm0 = out_lane && ok0, dm1 = out_lane && ok1;
  auto mdot = [&](cg_f4 a, cg_f4 b) {
    const cg_f2 p = cg_lo(a) * cg_lo(b), q = cg_hi(a) * cg_hi(b);
    return (dm0 ? p.x + p.y : 0.f) + (dm1 ? q.x + q.y : 0.f);
  };
  const cg_f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const int ns = r0 - 7, ne = r1 + 5;

  CgRaw SG[2];   // staged coefficient rows n+2, n+3
  cg_f4 PO[8];   // p_old of rows n-4 .. n+2
  cg_f4 RI[2];   // r_in of rows n-1, n
  cg_f4 XI[2];   // x of rows n-4, n-3
  if (live) {
    // rows ns .. ns+2 (coefficients), ns, ns+1 (p_old), ns (r_in)
    load_raw(ns, SG[0]);
    PO[0] = load_po(ns);
    PO[1] = load_po(ns + 1);
    RI[0] = load_rin(ns);
#pragma unroll
    for (int s = 2; s < 8; ++s) PO[s] = zero4;
    RI[1] = zero4;
    XI[0] = XI[1] = zero4;
  }
  float alpha = 0.f, beta = 0.f;
  if (cg_prologue<FIRST>(g, k, lds, &alpha, &beta)) return;

  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  if (live) {
    {
      // ring slot 0 <- row ns; slots 1..7 <- zero rows (read before written
      // only by stages whose rows lie above the band's valid region)
      put_rec(0, SG[0]);
      CgRaw zr;
      zr.wxu = zr.wyu = zr.wxv = zr.wyv = zr.a = zr.c = zr.d = cg_f2{0.f, 0.f};
#pragma unroll
      for (int s = 1; s < 8; ++s) put_rec(s, zr);
      load_raw(ns + 1, SG[1]);
      load_raw(ns + 2, SG[0]);
    }
    cg_f4 YR[4], G2[4], G1[4], PP[4], YQ[4], ZZ[2], V1[2];
#pragma unroll
    for (int s = 0; s < 4; ++s) YR[s] = G2[s] = G1[s] = PP[s] = YQ[s] = zero4;
    ZZ[0] = ZZ[1] = V1[0] = V1[1] = zero4;
    for (int n0 = ns; n0 <= ne; n0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int n = n0 + u;
        if (n > ne) break;
        // ring slots: row n + d lives in PO / LDS slot (u + d) & 7, in the
        // 4-rings at (u + d) & 3 and in the 2-rings at (u + d) & 1
#define S8(d) ((u + (d) + 16) & 7)
#define S4(d) ((u + (d) + 16) & 3)
#define S2(d) ((u + (d) + 16) & 1)
        // vertical weights of row n-7 (its slot is about to take row n+1)
        cg_f2 wy7[2];
        get_wy(S8(-7), wy7);
        put_rec(S8(1), SG[S2(1)]);
        load_raw(n + 3, SG[S2(1)]);
        PO[S8(2)] = load_po(n + 2);
        RI[S2(0)] = load_rin(n);
        XI[S2(-3)] = load_x(n - 3);
        // LDS records are read one stage ahead of their use (the ds_read
        // latency overlaps the previous stage's arithmetic)
        CgRec qn = get_rec(S8(-1));
        cg_f2 wn[2];
        get_wy(S8(-2), wn);
        // A) row n-1: r = r_in - alpha A p_old, y = D^-1 r
        {
          const CgRec q1 = qn;
          cg_f2 wu[2] = {wn[0], wn[1]};
          qn = get_rec(S8(-2));
          get_wy(S8(-3), wn);
          cg_f4 r = RI[S2(-1)];
          if (!FIRST) r -= alpha * (cgr_diag(q1, PO[S8(-1)]) - cgr_nsum(PO[S8(-2)], PO[S8(-1)], PO[S8(0)], q1, wu));
          const cg_f4 y = cgr_minv(q1, r);
          YR[S4(-1)] = y;
          const int o = n - 1;
          if (o >= r0 && o < r1) {
            cg_st4(rro, soff8 + (unsigned)o * rowb8, r);
            acc[4] += (double)mdot(r, r);
            acc[3] += (double)(c0 * mdot(r, y));
          }
        }
        // B) row n-2: g2 = c2 y + c3 D^-1 N y
        {
          const CgRec q2 = qn;
          cg_f2 wu[2] = {wn[0], wn[1]};
          qn = get_rec(S8(-3));
          get_wy(S8(-4), wn);
          const cg_f4 ny = cgr_nsum(YR[S4(-3)], YR[S4(-2)], YR[S4(-1)], q2, wu);
          G2[S4(-2)] = c2 * YR[S4(-2)] + c3 * cgr_minv(q2, ny);
        }
        // C) row n-3: g1 = c1 y + D^-1 N g2
        {
          const CgRec q3 = qn;
          cg_f2 wu[2] = {wn[0], wn[1]};
          qn = get_rec(S8(-4));
          get_wy(S8(-5), wn);
          const cg_f4 ng = cgr_nsum(G2[S4(-4)], G2[S4(-3)], G2[S4(-2)], q3, wu);
          G1[S4(-3)] = c1 * YR[S4(-3)] + cgr_minv(q3, ng);
        }
        // D) row n-4: z = c0 y + D^-1 N g1, p = z + beta p_old, x += alpha p_old
        {
          const CgRec q4 = qn;
          cg_f2 wu[2] = {wn[0], wn[1]};
          qn = get_rec(S8(-5));
          get_wy(S8(-6), wn);
          const cg_f4 ng = cgr_nsum(G1[S4(-5)], G1[S4(-4)], G1[S4(-3)], q4, wu);
          const cg_f4 yr = YR[S4(-4)];
          const cg_f4 z = c0 * yr + cgr_minv(q4, ng);
          cg_f4 p = FIRST ? z : z + beta * PO[S8(-4)];
          const int o = n - 4;
          const bool rv = (unsigned)o < (unsigned)H;
          if (!(rv && ok0)) { p.x = 0.f; p.y = 0.f; }
          if (!(rv && ok1)) { p.z = 0.f; p.w = 0.f; }
          PP[S4(-4)] = p;
          ZZ[S2(-4)] = z;
          if (o >= r0 && o < r1) {
            const unsigned so = soff8 + (unsigned)o * rowb8;
            cg_st4(rpn, so, p);
            cg_st4(rx, so, FIRST ? zero4 : XI[S2(-4)] + alpha * PO[S8(-4)]);
            acc[3] += (double)mdot(yr, ng);
          }
        }
        // E) row n-5: q = A p, y_q = D^-1 q
        {
          const CgRec q5 = qn;
          cg_f2 wu[2] = {wn[0], wn[1]};
          qn = get_rec(S8(-6));
          const cg_f4 pm = PP[S4(-5)];
          const cg_f4 q = cgr_diag(q5, pm) - cgr_nsum(PP[S4(-6)], pm, PP[S4(-4)], q5, wu);
          const cg_f4 yq = cgr_minv(q5, q);
          YQ[S4(-5)] = yq;
          const int o = n - 5;
          if (o >= r0 && o < r1) {
            acc[0] += (double)mdot(pm, q);
            acc[1] += (double)mdot(q, ZZ[S2(-5)]);
            acc[2] += (double)(c0 * mdot(q, yq));
          }
        }
        // F) row n-6: N y_q, v1 = D^-1 N y_q, T1..T3
        {
          const CgRec q6 = qn;
          const cg_f4 yq = YQ[S4(-6)];
          const cg_f4 ny = cgr_nsum(YQ[S4(-7)], yq, YQ[S4(-5)], q6, wy7);
          const cg_f4 v1 = cgr_minv(q6, ny);
          const cg_f4 vu = V1[S2(-7)];
          V1[S2(-6)] = v1;
          const int o = n - 6;
          if (o >= r0 && o < r1) {
            // edges to the left and above, counted by this (right / lower)
            // pixel: N v1 restricted to those edges
            const cg_f2 v0 = cg_lo(v1), vv1 = cg_hi(v1);
            const cg_f2 h0 = cg_left2(q6.wx[1]) * cg_left2(vv1) + wy7[0] * cg_lo(vu);
            const cg_f2 h1 = q6.wx[0] * v0 + wy7[1] * cg_hi(vu);
            const cg_f4 t = (c1 * yq + c2 * v1) * ny + (2.0f * c3) * v1 * cg_cat(h0, h1);
            acc[2] += (double)((dm0 ? t.x + t.y : 0.f) + (dm1 ? t.z + t.w : 0.f));
          }
        }
#undef S8
#undef S4
#undef S2
      }
    }
  }
  write_partials<5>(acc, g.part, lds);
}

// ---------------------------------------------------------------------------
// k_cg_small: a whole CG solve in ONE workgroup, for levels of at most
// CG_SMALL_PX pixels.  At the coarse pyramid levels a fused k_cgp launch is
// latency-bound (~23 us however few rows: its 7-stage row pipeline is walked
// by one wave per band), and a solve is one launch per iteration; here the
// whole solve is one launch.  Textbook preconditioned CG with the control
// flow of scipy.sparse.linalg.cg (base.py:116-136): x0 = 0, stop when
// ||r|| < rtol ||b|| before an iteration, at most maxiter iterations.
// Preconditioner as in the fused kernels: DEG 3 = k_cgp's Chebyshev
// polynomial in the 2x2 block-Jacobi splitting A = D - N (Horner, three
// neighbour sums), DEG 0 = D^-1 (2x2 blocks if BLOCK, else scipy's scalar
// Jacobi).  Vectors live in global memory (L2-resident at these sizes);
// sweeps are separated by workgroup barriers; reductions are fixed-order fp64.
#define CGS_BX 64
#define CGS_BY 16
#define CG_SMALL_PX 4096

struct CgSmallArgs {
  const float *coef;  // 7 planes, plane stride ps
  size_t ps;
  const float2 *b;
  float2 *x, *r, *p, *q, *y, *t;
  int H, W, P;
  double rtol;
  int maxiter;
  float poly[4];
  PcgState *st;
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
  int it = 0, done = 0;
  const float c0 = g.poly[0], c1 = g.poly[1], c2 = g.poly[2], c3 = g.poly[3];
  for (;; ++it) {
    if (rr == 0.0 && it == 0) { done = 3; break; }
    if (sqrt(rr) < atol) { done = 1; break; }
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
      CGS_FOR_PIXELS(H, W) {
        const size_t k = (size_t)i * P + j;
        g.y[k] = cgs_minv<BLOCK>(cf, ps, k, g.r[k]);
      }
      __syncthreads();
      CGS_FOR_PIXELS(H, W) {  // g2 = c2 y + c3 D^-1 N y
        const size_t k = (size_t)i * P + j;
        const float2 ny = cgs_minv<BLOCK>(cf, ps, k, cgs_nsum(cf, ps, g.y, i, j, H, W, P)), yk = g.y[k];
        g.t[k] = make_float2(c2 * yk.x + c3 * ny.x, c2 * yk.y + c3 * ny.y);
      }
      __syncthreads();
      CGS_FOR_PIXELS(H, W) {  // g1 = c1 y + D^-1 N g2
        const size_t k = (size_t)i * P + j;
        const float2 ng = cgs_minv<BLOCK>(cf, ps, k, cgs_nsum(cf, ps, g.t, i, j, H, W, P)), yk = g.y[k];
        g.q[k] = make_float2(c1 * yk.x + ng.x, c1 * yk.y + ng.y);
      }
      __syncthreads();
      CGS_FOR_PIXELS(H, W) {  // z = c0 y + D^-1 N g1
        const size_t k = (size_t)i * P + j;
        const float2 ng = cgs_minv<BLOCK>(cf, ps, k, cgs_nsum(cf, ps, g.q, i, j, H, W, P)), yk = g.y[k];
        const float2 z = make_float2(c0 * yk.x + ng.x, c0 * yk.y + ng.y), rk = g.r[k];
        g.t[k] = z;
        acc += (double)(rk.x * z.x + rk.y * z.y);
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
  }
}
template __global__ void k_cg_small<3, true>(CgSmallArgs);
template __global__ void k_cg_small<0, true>(CgSmallArgs);
template __global__ void k_cg_small<0, false>(CgSmallArgs);

// ---------------------------------------------------------------------------
// k_cgs: k_cgp's iteration (same preconditioner, same rho recurrence, same
// per-element arithmetic) with its pipeline stages split over the 4 waves of
// a block, which all work on ONE band:
//   wave 0: loads, coefficient records -> LDS ring, A) r, y of row n-1
//   wave 1: B) g2 of row n-3, C) g1 of row n-4
//   wave 2: D) z, p, x of row n-6, E) q, y_q of row n-7
//   wave 3: F) v1 and the T terms of row n-9
// with one block barrier per row step; rows cross waves through small LDS
// rings (y, g1, y_q; records in a 12-row ring), a wave's own rows stay in
// registers.  k_cgp gives each wave its own band and the whole pipeline, so
// a band of R rows costs R + 12 steps of all 6 stages per wave and its
// 32-KB record ring allows one wave per SIMD (R = 20 at 1080p: 1.6x the rows
// read); here 64 KB of LDS per block allow 2 blocks per CU (R = 39 at
// 1080p, 1.36x) and a step costs only the heaviest wave's share.
// Stage lags follow from one barrier per step: a stage reads rows of another
// wave produced at earlier steps; the band is walked for n in
// [r0 - 5, r1 + 8] so that every row a required stage reads was produced.
#define CGS_NREC 12

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
  const int lane = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(threadIdx.y), band = blockIdx.y;
  const int tid = lane + wid * 64;
  const int jc = blockIdx.x * PCG_SWP - 8 + 2 * lane;
  const bool ok0 = jc >= 0 && jc < W, ok1 = jc + 1 < W && jc >= 0;
  const bool out_lane = lane >= 4 && lane <= 59;
  const unsigned off4 = ok0 ? (unsigned)jc * 4u : CG_OOB, off8 = ok0 ? (unsigned)jc * 8u : CG_OOB;
  const unsigned soff8 = ok0 && out_lane ? (unsigned)jc * 8u : CG_OOB;
  const bool live = band < nbands;
  const int r0 = band * R, r1 = min(r0 + R, H);
  const float c0 = g.poly[0], c1 = g.poly[1], c2 = g.poly[2], c3 = g.poly[3];
  auto o4 = [&](int t) { return off4 + ((unsigned)t < (unsigned)H ? (unsigned)t * rowb4 : CG_ROW_OOB); };
  auto o8 = [&](int t) { return off8 + ((unsigned)t < (unsigned)H ? (unsigned)t * rowb8 : CG_ROW_OOB); };
  auto load_raw = [&](int t, CgRaw &c) {
    const unsigned v = o4(t);
    c.wxu = cg_mask1<ODD>(cg_ld2(rc, v, 0), ok1);
    c.wyu = cg_mask1<ODD>(cg_ld2(rc, v, ps4), ok1);
    c.wxv = cg_mask1<ODD>(cg_ld2(rc, v, 2 * ps4), ok1);
    c.wyv = cg_mask1<ODD>(cg_ld2(rc, v, 3 * ps4), ok1);
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
  auto load_x = [&](int t) {
    return (!FIRST && t >= r0 && t < r1) ? cg_mask1<ODD>(cg_ld4(rx, o8(t)), ok1) : cg_f4{0.f, 0.f, 0.f, 0.f};
  };
  const bool dm0 = out_lane && ok0, dm1 = out_lane && ok1;
  auto mdot = [&](cg_f4 a, cg_f4 b) {
    const cg_f2 p = cg_lo(a) * cg_lo(b), q = cg_hi(a) * cg_hi(b);
    return (dm0 ? p.x + p.y : 0.f) + (dm1 ? q.x + q.y : 0.f);
  };
  const cg_f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const int ns = r0 - 5, ne = r1 + 8;

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
  // wave 0: raw rows ns-2 .. ns+1, p_old rows ns-2 .. ns+1, r_in row ns-1
  // wave 2: p_old, x of row ns-6 (register rings indexed by (row - ns))
  CgRaw SG[4], SGp[2];
  cg_f4 PO[8], RI[2], PO2[2], XI[2];
  if (live && wid == 0) {
    load_raw(ns - 2, SGp[0]);
    load_raw(ns - 1, SGp[1]);
    load_raw(ns, SG[0]);
    load_raw(ns + 1, SG[1]);
#pragma unroll
    for (int m = -2; m <= 1; ++m) PO[m & 7] = load_po(ns + m);
    RI[1] = load_rin(ns - 1);
  }
  if (live && wid == 2) {
    PO2[0] = load_po(ns - 6);
    XI[0] = load_x(ns - 6);
  }
  float alpha = 0.f, beta = 0.f;
  if (cg_prologue<FIRST>(g, k, lds, &alpha, &beta)) return;

  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  if (live) {
    if (wid == 0) {
      put_rec(ns - 2, SGp[0]);
      put_rec(ns - 1, SGp[1]);
    }
    __syncthreads();
    // each wave runs its own role's loop (registers of one role only), one
    // block barrier per row step in every role (same step count)
#define CGS_STEPS(...)                                                    \
  for (int n0 = ns; n0 <= ne; n0 += 8) {                                  \
    _Pragma("unroll") for (int u = 0; u < 8; ++u) {                       \
      const int n = n0 + u;                                               \
      if (n > ne) break;                                                  \
      __VA_ARGS__                                                         \
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");              \
      __builtin_amdgcn_s_barrier();                                       \
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");              \
    }                                                                     \
  }
// register-ring index of row n + d: (u + d) mod ring size
#define R8(d) ((u + (d) + 16) & 7)
#define R4(d) ((u + (d) + 16) & 3)
#define R2(d) ((u + (d) + 16) & 1)
    if (wid == 0) {
      CGS_STEPS({
        load_raw(n + 2, SG[R4(2)]);
        PO[R8(2)] = load_po(n + 2);
        RI[R2(0)] = load_rin(n);
        put_rec(n, SG[R4(0)]);
        // A) row n-1: r = r_in - alpha A p_old, y = D^-1 r
        const CgRec q1 = get_rec(n - 1);
        cg_f2 wu[2];
        get_wy(n - 2, wu);
        cg_f4 r = RI[R2(-1)];
        if (!FIRST) r -= alpha * (cgr_diag(q1, PO[R8(-1)]) - cgr_nsum(PO[R8(-2)], PO[R8(-1)], PO[R8(0)], q1, wu));
        const cg_f4 y = cgr_minv(q1, r);
        s_y[(n - 1) & 7][lane] = make_float4(y.x, y.y, y.z, y.w);
        const int o = n - 1;
        if (o >= r0 && o < r1) {
          cg_st4(rro, soff8 + (unsigned)o * rowb8, r);
          acc[4] += (double)mdot(r, r);
          acc[3] += (double)(c0 * mdot(r, y));
        }
      })
    } else if (wid == 1) {
      cg_f4 G2[4] = {zero4, zero4, zero4, zero4};
      CGS_STEPS({
        // B) row n-3: g2 = c2 y + c3 D^-1 N y
        {
          const CgRec q2 = get_rec(n - 3);
          cg_f2 wu[2];
          get_wy(n - 4, wu);
          const float4 a = s_y[(n - 4) & 7][lane], b = s_y[(n - 3) & 7][lane], c = s_y[(n - 2) & 7][lane];
          const cg_f4 ym = {a.x, a.y, a.z, a.w}, y0 = {b.x, b.y, b.z, b.w}, yp = {c.x, c.y, c.z, c.w};
          const cg_f4 ny = cgr_nsum(ym, y0, yp, q2, wu);
          G2[R4(-3)] = c2 * y0 + c3 * cgr_minv(q2, ny);
        }
        // C) row n-4: g1 = c1 y + D^-1 N g2
        {
          const CgRec q3 = get_rec(n - 4);
          cg_f2 wu[2];
          get_wy(n - 5, wu);
          const float4 b = s_y[(n - 4) & 7][lane];
          const cg_f4 y0 = {b.x, b.y, b.z, b.w};
          const cg_f4 ng = cgr_nsum(G2[R4(-5)], G2[R4(-4)], G2[R4(-3)], q3, wu);
          st4(s_g1, n - 4, c1 * y0 + cgr_minv(q3, ng));
        }
      })
    } else if (wid == 2) {
      cg_f4 PP[4] = {zero4, zero4, zero4, zero4}, ZZ[2] = {zero4, zero4};
      CGS_STEPS({
        PO2[R2(-5)] = load_po(n - 5);
        XI[R2(-5)] = load_x(n - 5);
        // D) row n-6: z = c0 y + D^-1 N g1, p = z + beta p_old, x += alpha p_old
        {
          const CgRec q4 = get_rec(n - 6);
          cg_f2 wu[2];
          get_wy(n - 7, wu);
          const cg_f4 ng = cgr_nsum(ld4(s_g1, n - 7), ld4(s_g1, n - 6), ld4(s_g1, n - 5), q4, wu);
          const float4 b = s_y[(n - 6) & 7][lane];
          const cg_f4 yr = {b.x, b.y, b.z, b.w};
          const cg_f4 z = c0 * yr + cgr_minv(q4, ng);
          cg_f4 p = FIRST ? z : z + beta * PO2[R2(-6)];
          const int o = n - 6;
          const bool rv = (unsigned)o < (unsigned)H;
          if (!(rv && ok0)) { p.x = 0.f; p.y = 0.f; }
          if (!(rv && ok1)) { p.z = 0.f; p.w = 0.f; }
          PP[R4(-6)] = p;
          ZZ[R2(-6)] = z;
          if (o >= r0 && o < r1) {
            const unsigned so = soff8 + (unsigned)o * rowb8;
            cg_st4(rpn, so, p);
            cg_st4(rx, so, FIRST ? zero4 : XI[R2(-6)] + alpha * PO2[R2(-6)]);
            acc[3] += (double)mdot(yr, ng);
          }
        }
        // E) row n-7: q = A p, y_q = D^-1 q
        {
          const CgRec q5 = get_rec(n - 7);
          cg_f2 wu[2];
          get_wy(n - 8, wu);
          const cg_f4 pm = PP[R4(-7)];
          const cg_f4 q = cgr_diag(q5, pm) - cgr_nsum(PP[R4(-8)], pm, PP[R4(-6)], q5, wu);
          const cg_f4 yq = cgr_minv(q5, q);
          st4(s_yq, n - 7, yq);
          const int o = n - 7;
          if (o >= r0 && o < r1) {
            acc[0] += (double)mdot(pm, q);
            acc[1] += (double)mdot(q, ZZ[R2(-7)]);
            acc[2] += (double)(c0 * mdot(q, yq));
          }
        }
      })
    } else {
      cg_f4 V1[2] = {zero4, zero4};
      CGS_STEPS({
        // F) row n-9: N y_q, v1 = D^-1 N y_q, T1..T3
        const CgRec q6 = get_rec(n - 9);
        cg_f2 wy7[2];
        get_wy(n - 10, wy7);
        const cg_f4 yq = ld4(s_yq, n - 9);
        const cg_f4 ny = cgr_nsum(ld4(s_yq, n - 10), yq, ld4(s_yq, n - 8), q6, wy7);
        const cg_f4 v1 = cgr_minv(q6, ny);
        const cg_f4 vu = V1[R2(-10)];
        V1[R2(-9)] = v1;
        const int o = n - 9;
        if (o >= r0 && o < r1) {
          const cg_f2 v0 = cg_lo(v1), vv1 = cg_hi(v1);
          const cg_f2 h0 = cg_left2(q6.wx[1]) * cg_left2(vv1) + wy7[0] * cg_lo(vu);
          const cg_f2 h1 = q6.wx[0] * v0 + wy7[1] * cg_hi(vu);
          const cg_f4 t = (c1 * yq + c2 * v1) * ny + (2.0f * c3) * v1 * cg_cat(h0, h1);
          acc[2] += (double)((dm0 ? t.x + t.y : 0.f) + (dm1 ? t.z + t.w : 0.f));
        }
      })
    }
#undef R8
#undef R4
#undef R2
#undef CGS_STEPS
  }
  write_partials<5>(acc, g.part, lds);
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
