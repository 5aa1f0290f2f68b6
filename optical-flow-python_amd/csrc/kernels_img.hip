// kernels_img.hip — image-side kernels: colour conversion, global min/max,
// scaling, ROF structure-texture split, correlation, bilinear resize and the
// cubic B-spline prefilter.  All are HBM-streaming stencils (no MFMA).
#include "kernels.h"

// ---------------------------------------------------------------------------
// global min / max (scale_image, image_processing.py:6-26)
// mm[0] = ordered-uint min, mm[1] = ordered-uint max (init by k_mm_init)
__global__ void k_mm_init(uint32_t *mm, int n) {
  int t = threadIdx.x;
  if (t < n) { mm[2 * t] = 0xffffffffu; mm[2 * t + 1] = 0u; }
}

// min/max over `planes` pitched planes; one result pair per launch (slot)
__global__ void k_minmax(const float *__restrict__ a, int H, int W, int P, int planes, size_t plane_stride,
                         uint32_t *mm) {
  uint32_t lo = 0xffffffffu, hi = 0u;
  OF_FOR_PIXELS(H, W) {
    if (j < W)
      for (int c = 0; c < planes; ++c) {
        uint32_t o = f2ord(a[c * plane_stride + (size_t)i * P + j]);
        lo = min(lo, o);
        hi = max(hi, o);
      }
  }
  for (int off = 32; off > 0; off >>= 1) {
    lo = min(lo, (uint32_t)__shfl_down((int)lo, off, 64));
    hi = max(hi, (uint32_t)__shfl_down((int)hi, off, 64));
  }
  // one atomic pair per block (launched with <= 256 blocks): thousands of
  // same-address atomics from every wave serialise at the memory side
  __shared__ uint32_t s_lo[OF_BY], s_hi[OF_BY];
  if (threadIdx.x == 0) {
    s_lo[threadIdx.y] = lo;
    s_hi[threadIdx.y] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    for (int w = 1; w < OF_BY; ++w) {
      lo = min(lo, s_lo[w]);
      hi = max(hi, s_hi[w]);
    }
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
}

// x -> (x - lo) / (hi - lo) * (vhigh - vlow) + vlow, or the midpoint when hi == lo
__global__ void k_scale(float *__restrict__ a, int H, int W, int P, int planes, size_t plane_stride,
                        const uint32_t *mm, float vlow, float vhigh) {
  const float lo = ord2f(mm[0]), hi = ord2f(mm[1]);
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    for (int c = 0; c < planes; ++c) {
      float &x = a[c * plane_stride + (size_t)i * P + j];
      x = hi == lo ? (vlow + vhigh) * 0.5f : (x - lo) / (hi - lo) * (vhigh - vlow) + vlow;
    }
  }
}

// ---------------------------------------------------------------------------
// colour conversion (interface.py:74-141).  rgb: interleaved H x W x C dense.
// T = float (caller-converted frames) or uint8_t (frames uploaded as bytes)
template <typename TI>
__global__ void k_rgb_max(const TI *__restrict__ rgb, long n, uint32_t *mm) {
  uint32_t hi = 0u;
  for (long k = blockIdx.x * (long)blockDim.x + threadIdx.x; k < n; k += (long)gridDim.x * blockDim.x)
    hi = max(hi, f2ord((float)rgb[k]));
  for (int off = 32; off > 0; off >>= 1) hi = max(hi, (uint32_t)__shfl_down((int)hi, off, 64));
  __shared__ uint32_t s_hi[4];  // 256-thread blocks: one atomic per block
  if ((threadIdx.x & 63) == 0) s_hi[threadIdx.x >> 6] = hi;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&mm[1], max(max(s_hi[0], s_hi[1]), max(s_hi[2], s_hi[3])));
}

__device__ __forceinline__ float q_u8(float x) {
  float q = floorf(x + 0.5f);
  return fminf(fmaxf(q, 0.0f), 255.0f);
}

// gray (uint8 round trip) of both frames; Lab of frame 1 when lab != nullptr
template <typename TI>
__global__ void k_rgb_prep(const TI *__restrict__ rgb1, const TI *__restrict__ rgb2, int H, int W, int C,
                           float *gray, int P, size_t ps, float *lab, const uint32_t *mm_rgbmax) {
  const bool norm = ord2f(mm_rgbmax[1]) > 1.0f;
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    size_t k = (size_t)i * W + j, o = (size_t)i * P + j;
    if (C == 1) {
      gray[o] = (float)rgb1[k];
      gray[ps + o] = (float)rgb2[k];
      if (lab) lab[o] = (float)rgb1[k];
      continue;
    }
    const TI *a = rgb1 + 3 * k, *b = rgb2 + 3 * k;
    const float a0 = (float)a[0], a1 = (float)a[1], a2 = (float)a[2];
    gray[o] = floorf(0.2989f * q_u8(a0) + 0.5870f * q_u8(a1) + 0.1140f * q_u8(a2) + 0.5f);
    gray[ps + o] = floorf(0.2989f * q_u8((float)b[0]) + 0.5870f * q_u8((float)b[1]) + 0.1140f * q_u8((float)b[2]) + 0.5f);
    if (!lab) continue;
    float R = a0, G = a1, B = a2;
    if (norm) { R /= 255.0f; G /= 255.0f; B /= 255.0f; }
    const float T = 0.008856f;
    float X = (0.412453f * R + 0.357580f * G + 0.180423f * B) / 0.950456f;
    float Y = 0.212671f * R + 0.715160f * G + 0.072169f * B;
    float Z = (0.019334f * R + 0.119193f * G + 0.950227f * B) / 1.088754f;
    float Y3 = cbrtf(Y);
    float fX = X > T ? cbrtf(X) : 7.787f * X + 16.0f / 116.0f;
    float fY = Y > T ? Y3 : 7.787f * Y + 16.0f / 116.0f;
    float fZ = Z > T ? cbrtf(Z) : 7.787f * Z + 16.0f / 116.0f;
    lab[o] = Y > T ? 116.0f * Y3 - 16.0f : 903.3f * Y;
    lab[ps + o] = 500.0f * (fX - fY);
    lab[2 * ps + o] = 200.0f * (fY - fZ);
  }
}

// ---------------------------------------------------------------------------
// ROF primal-dual iteration (image_processing.py:86-136), one channel per
// blockIdx.z.  p: float2 {p_x, p_y} per pixel; ping-pong pin -> pout.
__device__ __forceinline__ float rof_div(const float2 *__restrict__ p, int i, int j, int P) {
  const float2 c = p[(size_t)i * P + j];
  float d = j > 0 ? c.x - p[(size_t)i * P + j - 1].x : c.x;
  d += i > 0 ? c.y - p[(size_t)(i - 1) * P + j].y : c.y;
  return d;
}

// ROF_K primal-dual iterations per launch (temporal blocking).  A block of
// 4 waves owns a ROF_TW x ROF_TH tile of one channel plus a ROF_K-wide halo:
// lane = column (ROF_RW = 64 = ROF_TW + 2 ROF_K), wave w = ROF_RPW
// consecutive rows, held in registers.  One iteration of a pixel's p reads
// p only at Chebyshev distance <= 1, so after `iters` <= ROF_K iterations the
// tile is exact; HBM traffic is one read of im + p and one write of p per
// launch instead of per iteration.  Horizontal neighbours are DPP lane
// shifts, vertical ones registers; only the rows at a wave boundary go
// through LDS (two barriers per iteration).  Per iteration:
//   u = im + theta div p   (div: backward differences, term dropped at
//                           image column / row 0)
//   p <- (p + delta grad u) / max(1, |.|)   (grad 0 at the last column / row)
// (image_processing.py:104-127).  Pixels outside the image hold p = im = 0
// and are never read by pixels inside it.  1 / max(1, |.|) is an rsq.
#define ROF_RW 64
#define ROF_K 8
#define ROF_TW (ROF_RW - 2 * ROF_K)
#define ROF_RPW 32
#define ROF_TH (4 * ROF_RPW - 2 * ROF_K)
__device__ __forceinline__ float rof_from_left(float v) {  // lane l <- lane l-1, lane 0 <- 0
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float rof_from_right(float v) {  // lane l <- lane l+1, lane 63 <- 0
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}
__global__ __launch_bounds__(256) void k_rof_iters(const float *__restrict__ im, const float2 *__restrict__ pin,
                                                   float2 *__restrict__ pout, int H, int W, int P, size_t ps,
                                                   float theta, float delta, int iters) {
  __shared__ float s_py[4][64], s_u[4][64];  // wave-boundary rows: p_y of the last, u of the first
  // XCD-aware tile order (common.h: of_xcd_tile): each XCD a contiguous run
  // of the (frame, row, column) tiles, so the 8-pixel halos two neighbouring
  // tiles both read meet in one L2 instead of being fetched twice
  const int gx = gridDim.x, gxy = gridDim.x * gridDim.y;
  const int t = of_xcd_tile(blockIdx.x + gx * blockIdx.y + gxy * blockIdx.z, gxy * gridDim.z);
  const int bz = t / gxy, by = (t - bz * gxy) / gx, bx = t - bz * gxy - by * gx;
  im += bz * ps;
  pin += bz * ps;
  pout += bz * ps;
  const int lane = threadIdx.x, w = __builtin_amdgcn_readfirstlane(threadIdx.y);
  const int gj = bx * ROF_TW - ROF_K + lane;
  const int gr0 = by * ROF_TH - ROF_K + w * ROF_RPW;  // image row of the wave's first row
  const bool colin = (unsigned)gj < (unsigned)W, left = gj > 0, right = gj < W - 1;
  float I[ROF_RPW], U[ROF_RPW];
  float2 Q[ROF_RPW];
#pragma unroll
  for (int r = 0; r < ROF_RPW; ++r) {
    const int gi = gr0 + r;
    const bool in = colin && (unsigned)gi < (unsigned)H;
    const size_t k = (size_t)gi * P + gj;
    I[r] = in ? im[k] : 0.0f;
    Q[r] = in ? pin[k] : make_float2(0.0f, 0.0f);
  }
  for (int it = 0; it < iters; ++it) {
    s_py[w][lane] = Q[ROF_RPW - 1].y;
    __syncthreads();
    float pya = w > 0 ? s_py[w - 1][lane] : 0.0f;  // p_y of the row above the wave's first row
#pragma unroll
    for (int r = 0; r < ROF_RPW; ++r) {
      const float2 q = Q[r];
      const float pl = rof_from_left(q.x);
      float d = left ? q.x - pl : q.x;
      d += gr0 + r > 0 ? q.y - pya : q.y;
      U[r] = I[r] + theta * d;
      pya = q.y;
    }
    s_u[w][lane] = U[0];
    __syncthreads();
    const float ub = w < 3 ? s_u[w + 1][lane] : 0.0f;  // u of the row below the wave's last row
#pragma unroll
    for (int r = 0; r < ROF_RPW; ++r) {
      const float u = U[r], ur = rof_from_right(u), ud = r + 1 < ROF_RPW ? U[r + 1] : ub;
      const float gx = right ? ur - u : 0.0f;
      const float gy = gr0 + r < H - 1 ? ud - u : 0.0f;
      const float a = Q[r].x + delta * gx, b = Q[r].y + delta * gy;
      const float s2 = a * a + b * b;
      const float inv = s2 > 1.0f ? __builtin_amdgcn_rsqf(s2) : 1.0f;
      Q[r] = make_float2(a * inv, b * inv);
    }
  }
  if (lane >= ROF_K && lane < ROF_K + ROF_TW && colin) {
#pragma unroll
    for (int r = 0; r < ROF_RPW; ++r) {
      const int gi = gr0 + r, tr = w * ROF_RPW + r;  // row inside the block's region
      if (tr >= ROF_K && tr < ROF_K + ROF_TH && gi < H) pout[(size_t)gi * P + gj] = Q[r];
    }
  }
}

// texture = im_norm - alp * (im_norm + theta div p)
__global__ void k_rof_final(const float *__restrict__ im, const float2 *__restrict__ p, float *__restrict__ out,
                            int H, int W, int P, size_t ps, float theta, float alp) {
  im += blockIdx.z * ps;
  p += blockIdx.z * ps;
  out += blockIdx.z * ps;
  OF_FOR_PIXELS_XCD(H, W) {
    if (j >= W) continue;
    size_t k = (size_t)i * P + j;
    out[k] = im[k] - alp * (im[k] + theta * rof_div(p, i, j, P));
  }
}

// ---------------------------------------------------------------------------
// scipy.ndimage.correlate(mode='reflect') with an odd kh x kw kernel, per plane z
__global__ void k_correlate(const float *__restrict__ in, float *__restrict__ out, int H, int W, int P, size_t ps,
                            Taps t) {
  in += blockIdx.z * ps;
  out += blockIdx.z * ps;
  const int ch = t.kh / 2, cw = t.kw / 2;
  OF_FOR_PIXELS_XCD(H, W) {
    if (j >= W) continue;
    float s = 0.0f;
    for (int a = 0; a < t.kh; ++a) {
      const float *row = in + (size_t)ext_reflect(i + a - ch, H) * P;
      for (int b = 0; b < t.kw; ++b) {
        float w = t.w[a * t.kw + b];
        if (w != 0.0f) s += w * row[ext_reflect(j + b - cw, W)];
      }
    }
    out[(size_t)i * P + j] = s;
  }
}

// the same with the kernel size fixed at compile time (taps unrolled into
// registers) and one-fold reflection, valid while the radius is below the
// plane size (host-checked): no integer modulo per tap
__device__ __forceinline__ int refl1(int i, int n) { return i < 0 ? -i - 1 : (i >= n ? 2 * n - 1 - i : i); }
template <int KH, int KW>
__global__ __launch_bounds__(OF_BX *OF_BY) void k_correlate_k(const float *__restrict__ in, float *__restrict__ out,
                                                             int H, int W, int P, size_t ps, Taps t) {
  in += blockIdx.z * ps;
  out += blockIdx.z * ps;
  constexpr int ch = KH / 2, cw = KW / 2;
  OF_FOR_PIXELS_XCD(H, W) {
    if (j >= W) continue;
    int cols[KW];
#pragma unroll
    for (int b = 0; b < KW; ++b) cols[b] = refl1(j + b - cw, W);
    float s = 0.0f;
#pragma unroll
    for (int a = 0; a < KH; ++a) {
      const float *row = in + (size_t)refl1(i + a - ch, H) * P;
#pragma unroll
      for (int b = 0; b < KW; ++b) {
        const float w = t.w[a * KW + b];
        if (w != 0.0f) s += w * row[cols[b]];
      }
    }
    out[(size_t)i * P + j] = s;
  }
}

// _matlab_imresize_bilinear / resample_flow: source coordinate
// (o + 0.5) * (H / nH) - 0.5 clipped to [0, H-1], bilinear, times `mult`.
template <typename T>
__global__ void k_resize(const T *__restrict__ in, int H, int W, int P, size_t ps, T *__restrict__ out, int nH, int nW,
                         int nP, size_t nps, float mult) {
  in += blockIdx.z * ps;
  out += blockIdx.z * nps;
  const float sy = (float)H / (float)nH, sx = (float)W / (float)nW;
  const int j = blockIdx.x * OF_BX + threadIdx.x;
  if (j >= nW) return;
  float c = fminf(fmaxf((j + 0.5f) * sx - 0.5f, 0.0f), (float)(W - 1));
  int j0 = (int)floorf(c);
  float fc = c - j0;
  int j1 = min(j0 + 1, W - 1);
  for (int o = blockIdx.y * OF_BY + threadIdx.y; o < nH; o += gridDim.y * OF_BY) {
    float r = fminf(fmaxf((o + 0.5f) * sy - 0.5f, 0.0f), (float)(H - 1));
    int i0 = (int)floorf(r);
    float fr = r - i0;
    int i1 = min(i0 + 1, H - 1);
    const T *r0 = in + (size_t)i0 * P, *r1 = in + (size_t)i1 * P;
    T v = (1.0f - fr) * ((1.0f - fc) * r0[j0] + fc * r0[j1]) + fr * ((1.0f - fc) * r1[j0] + fc * r1[j1]);
    out[(size_t)o * nP + j] = mult * v;
  }
}
template __global__ void k_resize<float>(const float *, int, int, int, size_t, float *, int, int, int, size_t, float);
template __global__ void k_resize<float2>(const float2 *, int, int, int, size_t, float2 *, int, int, int, size_t,
                                          float);

// ---------------------------------------------------------------------------
// cubic B-spline prefilter with mirror boundary = the symmetric IIR
// 6 / (z + 4 + 1/z) realised as a truncated FIR h[k] = c0 * zp^|k|,
// zp = sqrt(3) - 2, c0 = -6 zp / (1 - zp^2), |k| <= OF_BSPL_K (zp^16 ~ 7e-10)
__global__ void k_bspline_rows(const float *__restrict__ in, float *__restrict__ out, int H, int W, int P, size_t ps,
                               BsplTaps t) {
  in += blockIdx.z * ps;
  out += blockIdx.z * ps;
  OF_FOR_PIXELS_XCD(H, W) {
    if (j >= W) continue;
    const float *row = in + (size_t)i * P;
    float s = t.h[0] * row[j];
    for (int k = 1; k <= OF_BSPL_K; ++k) s += t.h[k] * (row[ext_mirror(j - k, W)] + row[ext_mirror(j + k, W)]);
    out[(size_t)i * P + j] = s;
  }
}
__global__ void k_bspline_cols(const float *__restrict__ in, float *__restrict__ out, int H, int W, int P, size_t ps,
                               BsplTaps t) {
  in += blockIdx.z * ps;
  out += blockIdx.z * ps;
  OF_FOR_PIXELS_XCD(H, W) {
    if (j >= W) continue;
    float s = t.h[0] * in[(size_t)i * P + j];
    for (int k = 1; k <= OF_BSPL_K; ++k)
      s += t.h[k] * (in[(size_t)ext_mirror(i - k, H) * P + j] + in[(size_t)ext_mirror(i + k, H) * P + j]);
    out[(size_t)i * P + j] = s;
  }
}

// ---------------------------------------------------------------------------
// layout converters between dense planar host images and pitched device data
__global__ void k_planar2_to_f2(const float *__restrict__ a, float2 *__restrict__ out, int H, int W, int P,
                                size_t dense_ps) {
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    size_t k = (size_t)i * W + j;
    out[(size_t)i * P + j] = make_float2(a[k], a[dense_ps + k]);
  }
}
__global__ void k_f2_to_planar2(const float2 *__restrict__ in, float *__restrict__ a, int H, int W, int P,
                                size_t dense_ps) {
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    size_t k = (size_t)i * W + j;
    float2 v = in[(size_t)i * P + j];
    a[k] = v.x;
    a[dense_ps + k] = v.y;
  }
}
__global__ void k_fill_f2(float2 *out, int H, int W, int P, float2 v) {
  OF_FOR_PIXELS(H, W) {
    if (j < W) out[(size_t)i * P + j] = v;
  }
}

// out = a - alp * b per plane (fc pre-filter)
__global__ void k_sub_scaled(const float *__restrict__ a, const float *__restrict__ b, float alp,
                             float *__restrict__ out, int H, int W, int P, size_t ps) {
  a += blockIdx.z * ps;
  b += blockIdx.z * ps;
  out += blockIdx.z * ps;
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    out[k] = a[k] - alp * b[k];
  }
}

// ---------------------------------------------------------------------------
// Middlebury flow colour coding (viz/flow_color.py:43-107; SURVEY.md §8f row
// 4).  One pass reduces the largest known radius, one maps each pixel through
// the 55-bin wheel.  The arithmetic follows numpy's dtype rules step by step,
// so the uint8 image equals the reference's: T = the flow's dtype for
// the normalisation, the radius, atan2(-v, -u) / pi and fk = (a + 1) / 2 * 54;
// f = fk - k0 and the colour blend in float64 (float32 - int64 promotes).  No
// contraction into fma: numpy rounds every product and sum on its own.
struct ColorWheel {
  unsigned char w[55 * 3];  // make_colorwheel (flow_color.py:5-40), RGB per bin
};

template <typename T> struct OrdBits;
template <> struct OrdBits<float> {
  using U = unsigned int;
  static __device__ U of(float x) { return __float_as_uint(x); }
  static __device__ float to(U b) { return __uint_as_float(b); }
};
template <> struct OrdBits<double> {
  using U = unsigned long long;
  static __device__ U of(double x) { return (U)__double_as_longlong(x); }
  static __device__ double to(U b) { return __longlong_as_double((long long)b); }
};

// largest sqrt(u^2 + v^2) over pixels with |u|, |v| <= 1e9 (flow_color.py:92-98);
// radii are >= 0, so their bit patterns order like the values (*mx starts at 0)
template <typename T>
__global__ void k_flow_rad_max(const T *__restrict__ flow, long n, typename OrdBits<T>::U *mx) {
#pragma clang fp contract(off)
  using U = typename OrdBits<T>::U;
  U best = 0;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < n; p += (long)gridDim.x * blockDim.x) {
    const T u = flow[2 * p], v = flow[2 * p + 1];
    if (fabs(u) > (T)1e9 || fabs(v) > (T)1e9) continue;
    const T r = sqrt(u * u + v * v);
    const U b = OrdBits<T>::of(r);
    best = b > best ? b : best;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const U o = __shfl_down(best, off, 64);
    best = o > best ? o : best;
  }
  if ((threadIdx.x & 63) == 0) atomicMax(mx, best);
}

// max_rad = max(max_rad, 1e-8) (flow_color.py:100) in T: the fixed max_flow
// (fixed > 0) or the reduced radius
template <typename T>
__device__ __forceinline__ T color_max_rad(const typename OrdBits<T>::U *mx, double fixed) {
  if (fixed > 0) return (T)(fixed > 1e-8 ? fixed : 1e-8);
  const T r = OrdBits<T>::to(*mx);
  return (T)1e-8 > r ? (T)1e-8 : r;
}

template <typename T>
__device__ __forceinline__ T color_atan2(T y, T x);
// float32: numpy's float32 arctan2 on the host is a vector-library routine
// (not correctly rounded, and CPU-dependent); the device rounds the float64
// atan2 to float32, the correctly rounded value (tests/test_gpu_viz.py states
// what that leaves)
template <> __device__ __forceinline__ float color_atan2<float>(float y, float x) {
  return (float)atan2((double)y, (double)x);
}
template <> __device__ __forceinline__ double color_atan2<double>(double y, double x) { return atan2(y, x); }

template <typename T>
__global__ void k_flow_color(const T *__restrict__ flow, long n, const typename OrdBits<T>::U *mx, double fixed,
                             ColorWheel cw, unsigned char *__restrict__ out) {
#pragma clang fp contract(off)
  const T mr = color_max_rad<T>(mx, fixed);
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < n; p += (long)gridDim.x * blockDim.x) {
    T u = flow[2 * p], v = flow[2 * p + 1];
    unsigned char rgb[3] = {0, 0, 0};
    if (!(fabs(u) > (T)1e9 || fabs(v) > (T)1e9)) {  // unknown flow stays black (:105)
      u = u / mr;
      v = v / mr;
      const T rad = sqrt(u * u + v * v);
      const T a = color_atan2<T>(-v, -u) / (T)3.141592653589793;
      const T fk = (a + (T)1) / (T)2 * (T)54;
      const int k0 = (int)floor(fk);
      const int k1 = k0 + 1 == 55 ? 0 : k0 + 1;
      const double f = (double)fk - (double)k0;
      for (int c = 0; c < 3; ++c) {
        double col = (double)cw.w[3 * k0 + c] / 255.0 * (1.0 - f) + (double)cw.w[3 * k1 + c] / 255.0 * f;
        col = 1.0 - (double)rad * (1.0 - col);
        if (rad > (T)1) col = col * 0.75;
        col = col < 0.0 ? 0.0 : (col > 1.0 ? 1.0 : col);
        rgb[c] = (unsigned char)floor(255.0 * col);
      }
    }
    out[3 * p] = rgb[0];
    out[3 * p + 1] = rgb[1];
    out[3 * p + 2] = rgb[2];
  }
}
