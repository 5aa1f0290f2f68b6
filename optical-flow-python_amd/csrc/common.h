// common.h — shared device helpers for liboptflow (gfx950 / CDNA4).
//
// Data layout in HBM (DESIGN.md §"Data layout"): every image plane is fp32
// row-major with a row pitch padded to a multiple of 64 floats (256 B), so a
// wave64 reads one aligned 256-B row segment per plane.  Flow-like vector
// fields (uv, PCG vectors) are float2 {u, v} per pixel with the same pitch.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "optflow.h"

#define OF_WAVE 64
#define OF_BX 64  // block x = one wave across a row
#define OF_BY 4   // 4 rows per block -> 256 threads

static inline int of_pitch(int W) { return (W + 63) & ~63; }

// ---- boundary extensions -------------------------------------------------
// scipy.ndimage mode='reflect' (half-sample symmetric: d c b a | a b c d)
__device__ __forceinline__ int ext_reflect(int i, int n) {
  if (n == 1) return 0;
  int p = 2 * n;
  i %= p;
  if (i < 0) i += p;
  return i < n ? i : p - 1 - i;
}
// np.pad 'reflect' / scipy 'mirror' (whole-sample: d c b | a b c d)
__device__ __forceinline__ int ext_mirror(int i, int n) {
  if (n == 1) return 0;
  int p = 2 * (n - 1);
  i %= p;
  if (i < 0) i += p;
  return i < n ? i : p - i;
}
__device__ __forceinline__ int clampi(int i, int lo, int hi) { return i < lo ? lo : (i > hi ? hi : i); }

// ---- robust penalty weights rho'(x)/x (penalties.py d_type == 2) ---------
struct PenF {
  int kind;
  float p0, p1;
  double d0, d1;  // the same parameters unrounded (pen_w_f64)
};

__host__ static inline PenF to_penf(const of_penalty &p) {
  PenF q;
  q.kind = p.kind;
  q.p0 = (float)p.p0;
  q.p1 = (float)p.p1;
  q.d0 = p.p0;
  q.d1 = p.p1;
  return q;
}

// rho'(x)/x per kind (penalties.py d_type == 2); pen_k<K> picks one at
// compile time (the assembly kernels specialised on the method's penalty
// kinds), pen_w at run time -- the same arithmetic either way
// OF_WARP_NOCONTRACT (default 1): no fma contraction in the warp / weight /
// assembly arithmetic, so the fused warp + assembly and the two-kernel form
// round every product and sum alike and assemble the same system bitwise
// (left to the compiler the two forms contracted different products; round
// 6, profiles/r6k: the smoke pair's mean |uv - oracle| 3.69e-3 -> 6.7e-4,
// every parity test green, -0.7 % pairs/s)
#ifndef OF_WARP_NOCONTRACT
#define OF_WARP_NOCONTRACT 1
#endif
#if OF_WARP_NOCONTRACT
#define OF_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define OF_NOCONTRACT
#endif
__device__ __forceinline__ float pen_quad(const PenF &p, float) { return 2.0f / (p.p0 * p.p0); }
__device__ __forceinline__ float pen_lorentz(const PenF &p, float x) {
  OF_NOCONTRACT return 2.0f / (2.0f * p.p0 * p.p0 + x * x); }
__device__ __forceinline__ float pen_charb(const PenF &p, float x) {
  OF_NOCONTRACT
  float s2 = p.p0 * p.p0, t = x / s2;
  return 1.0f / (s2 * sqrtf(1.0f + t * t));
}
// (sigma^2 + x^2)^(a-1) as exp2((a-1) log2(.)): the base is a normal
// positive float (sigma^2 + x^2 >= sigma^2), so the hardware v_log_f32 /
// v_exp_f32 pair (~1 ulp each) replaces the ~30-instruction general powf
__device__ __forceinline__ float pen_gcharb(const PenF &p, float x) {
  OF_NOCONTRACT
  return 2.0f * p.p1 * __builtin_amdgcn_exp2f((p.p1 - 1.0f) * __builtin_amdgcn_logf(p.p0 * p.p0 + x * x));
}
__device__ __forceinline__ float pen_w(const PenF &p, float x) {
  OF_NOCONTRACT
  switch (p.kind) {
    case OF_PEN_QUADRATIC: return pen_quad(p, x);
    case OF_PEN_LORENTZIAN: return pen_lorentz(p, x);
    case OF_PEN_CHARBONNIER: return pen_charb(p, x);
    case OF_PEN_GEN_CHARBONNIER: return pen_gcharb(p, x);
    case OF_PEN_GEMAN_MCCLURE: {
      float s2 = p.p0 * p.p0, d = s2 + x * x;
      return 2.0f * s2 / (d * d);
    }
    case OF_PEN_HUBER: {
      float s2 = p.p0 * p.p0, ax = fabsf(x);
      return ax <= s2 ? 2.0f : 2.0f * s2 / fmaxf(ax, 1e-30f);
    }
    case OF_PEN_TUKEY: {
      float s2 = p.p0 * p.p0, om = 1.0f - x * x / s2;
      return fabsf(x) <= p.p0 ? 2.0f * om * om / s2 : 0.0f;
    }
    case OF_PEN_GAUSSIAN: return 1.0f / (p.p0 * p.p0);
    case OF_PEN_TDIST:
    case OF_PEN_TDIST_UNNORM: return (p.p0 + 1.0f) / (p.p1 * p.p1 * p.p0 + x * x);
    default: return p.p0;  // OF_PEN_CONST
  }
}
template <int K>
__device__ __forceinline__ float pen_k(const PenF &p, float x) {
  OF_NOCONTRACT
  if constexpr (K == OF_PEN_QUADRATIC) return pen_quad(p, x);
  else if constexpr (K == OF_PEN_LORENTZIAN) return pen_lorentz(p, x);
  else if constexpr (K == OF_PEN_CHARBONNIER) return pen_charb(p, x);
  else if constexpr (K == OF_PEN_GEN_CHARBONNIER) return pen_gcharb(p, x);
  else if constexpr (K == OF_PEN_CONST) return p.p0;
  else return pen_w(p, x);
}

// rho'(x)/x in fp64 (penalties.py d_type == 2, the reference's own float64
// formulas): the assembly of ill-conditioned systems (k_flow_operator_f64)
__device__ __forceinline__ double pen_w_f64(const PenF &p, double x) {
  switch (p.kind) {
    case OF_PEN_QUADRATIC: return 2.0 / (p.d0 * p.d0);
    case OF_PEN_LORENTZIAN: return 2.0 / (2.0 * p.d0 * p.d0 + x * x);
    case OF_PEN_CHARBONNIER: {
      const double s2 = p.d0 * p.d0, t = x / s2;
      return 1.0 / (s2 * sqrt(1.0 + t * t));
    }
    case OF_PEN_GEN_CHARBONNIER: return 2.0 * p.d1 * pow(p.d0 * p.d0 + x * x, p.d1 - 1.0);
    case OF_PEN_GEMAN_MCCLURE: {
      const double s2 = p.d0 * p.d0, d = s2 + x * x;
      return 2.0 * s2 / (d * d);
    }
    case OF_PEN_HUBER: {
      const double s2 = p.d0 * p.d0, ax = fabs(x);
      return ax <= s2 ? 2.0 : 2.0 * s2 / fmax(ax, 1e-300);
    }
    case OF_PEN_TUKEY: {
      const double s2 = p.d0 * p.d0, om = 1.0 - x * x / s2;
      return fabs(x) <= p.d0 ? 2.0 * om * om / s2 : 0.0;
    }
    case OF_PEN_GAUSSIAN: return 1.0 / (p.d0 * p.d0);
    case OF_PEN_TDIST:
    case OF_PEN_TDIST_UNNORM: return (p.d0 + 1.0) / (p.d1 * p.d1 * p.d0 + x * x);
    default: return p.d0;  // OF_PEN_CONST
  }
}

// ---- order-preserving float <-> uint32 (sorting, atomic min/max) ----------
__device__ __forceinline__ uint32_t f2ord(float f) {
  uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t o) {
  uint32_t b = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
  return __uint_as_float(b);
}

// ---- reductions -----------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// Sum NV doubles over the block (256 threads max); result valid in thread 0.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double *lds /* NV*16 */) {
  const int tid = threadIdx.x + threadIdx.y * blockDim.x;
  const int nw = (blockDim.x * blockDim.y + 63) / 64;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
  if ((tid & 63) == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) lds[k * 16 + (tid >> 6)] = v[k];
  __syncthreads();
  if (tid == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double s = 0;
      for (int w = 0; w < nw; ++w) s += lds[k * 16 + w];
      v[k] = s;
    }
}

// ---- launch geometry: 64x4 blocks, grid-stride over row groups ----------
struct Grid2 {
  dim3 grid, block;
  int nblocks;
};
static inline Grid2 grid2(int H, int W, int max_blocks = 2048) {
  Grid2 g;
  g.block = dim3(OF_BX, OF_BY, 1);
  int gx = (W + OF_BX - 1) / OF_BX;
  int gy = (H + OF_BY - 1) / OF_BY;
  int cap = max_blocks / gx;
  if (cap < 1) cap = 1;
  if (gy > cap) gy = cap;
  g.grid = dim3(gx, gy, 1);
  g.nblocks = gx * gy;
  return g;
}

// pixel loop of a grid2 launch: for (i...) rows, j column
#define OF_FOR_PIXELS(H, W)                                        \
  const int j = blockIdx.x * OF_BX + threadIdx.x;                  \
  for (int i = blockIdx.y * OF_BY + threadIdx.y; i < (H); i += gridDim.y * OF_BY)

// The same loop with an XCD-aware block order, for stencil / gather kernels
// whose blocks read their neighbours' rows: workgroups b, b + 8, b + 16 ...
// run on one XCD (one L2), so each XCD gets a contiguous range of the grid's
// row-major blocks and vertically / horizontally adjacent blocks share their
// halo rows in one L2 instead of fetching them from HBM twice.  A permutation
// of the blocks: every pixel is still visited once, by one thread.
__device__ __forceinline__ int of_xcd_tile(int lin, int nt) {
  const int xcd = lin & 7;
  return xcd * (nt >> 3) + min(xcd, nt & 7) + (lin >> 3);
}
#define OF_FOR_PIXELS_XCD(H, W)                                                                       \
  const int of_t_ = of_xcd_tile(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);         \
  const int of_by_ = of_t_ / (int)gridDim.x;                                                          \
  const int j = (of_t_ - of_by_ * (int)gridDim.x) * OF_BX + threadIdx.x;                              \
  for (int i = of_by_ * OF_BY + threadIdx.y; i < (H); i += gridDim.y * OF_BY)
