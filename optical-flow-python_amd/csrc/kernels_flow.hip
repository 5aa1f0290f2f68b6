// kernels_flow.hip — the per-warping-iteration kernels of the IRLS loop:
// warp + derivatives, matrix-free flow-operator assembly, update/clip +
// occlusion, 5x5 median and the occlusion-weighted colour-guided weighted
// median.  See DESIGN.md for the roofline of each.
#include "kernels.h"

// ---------------------------------------------------------------------------
// cubic Hermite basis (tensor-product form of derivatives.py:7-24's
// 16x16 bicubic coefficient matrix)
__device__ __forceinline__ void hermite(float t, float h[4], float dh[4]) {
  float t2 = t * t, t3 = t2 * t;
  h[0] = 2.0f * t3 - 3.0f * t2 + 1.0f;
  h[1] = -2.0f * t3 + 3.0f * t2;
  h[2] = t3 - 2.0f * t2 + t;
  h[3] = t3 - t2;
  dh[0] = 6.0f * t2 - 6.0f * t;
  dh[1] = -6.0f * t2 + 6.0f * t;
  dh[2] = 3.0f * t2 - 4.0f * t + 1.0f;
  dh[3] = 3.0f * t2 - 2.0f * t;
}

__device__ __forceinline__ float bspline3(float t) {
  t = fabsf(t);
  if (t < 1.0f) return 2.0f / 3.0f - t * t + 0.5f * t * t * t;
  if (t < 2.0f) {
    float s = 2.0f - t;
    return s * s * s * (1.0f / 6.0f);
  }
  return 0.0f;
}

// partial_deriv (derivatives.py:148-296) for one pixel and all channels.
// (x2, y2) are the 1-based warped coordinates.
template <int INTERP>
__device__ __forceinline__ void warp_pixel(const DerivArgs &d, int H, int W, int P, size_t ps, int i, int j, float x2,
                                           float y2, float *it, float *ix, float *iy) {
  const size_t k = (size_t)i * P + j;
  if (INTERP == OF_INTERP_BICUBIC) {
    float fx = floorf(x2), fy = floorf(y2);
    bool oob = (fx < 1.0f) || (fx + 1.0f > (float)W) || (fy < 1.0f) || (fy + 1.0f > (float)H) || !(x2 == x2) ||
               !(y2 == y2);
    int fx0 = (int)fminf(fmaxf(fx, 1.0f), (float)W) - 1, cx0 = (int)fminf(fmaxf(fx + 1.0f, 1.0f), (float)W) - 1;
    int fy0 = (int)fminf(fmaxf(fy, 1.0f), (float)H) - 1, cy0 = (int)fminf(fmaxf(fy + 1.0f, 1.0f), (float)H) - 1;
    float ax = oob ? 0.0f : x2 - fx, ay = oob ? 0.0f : y2 - fy;
    float hx[4], dhx[4], hy[4], dhy[4];
    hermite(ax, hx, dhx);
    hermite(ay, hy, dhy);
    const size_t cs[4] = {(size_t)fy0 * P + fx0, (size_t)fy0 * P + cx0, (size_t)cy0 * P + fx0, (size_t)cy0 * P + cx0};
    for (int c = 0; c < d.nc; ++c) {
      const size_t o = c * ps;
      float v = 0.0f, vx = 0.0f, vy = 0.0f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int xi = q & 1, yi = q >> 1;
        const float z = d.I2[o + cs[q]], dx = d.A[o + cs[q]], dy = d.B[o + cs[q]], dxy = d.Cc[o + cs[q]];
        const float gx = hx[xi], gy = hy[yi], sx = hx[2 + xi], sy = hy[2 + yi];
        v += gx * gy * z + sx * gy * dx + gx * sy * dy + sx * sy * dxy;
        vx += dhx[xi] * gy * z + dhx[2 + xi] * gy * dx + dhx[xi] * sy * dy + dhx[2 + xi] * sy * dxy;
        vy += gx * dhy[yi] * z + sx * dhy[yi] * dx + gx * dhy[2 + yi] * dy + sx * dhy[2 + yi] * dxy;
      }
      if (oob) {
        it[c] = ix[c] = iy[c] = 0.0f;
      } else {
        it[c] = v - d.I1[o + k];
        ix[c] = d.blend * vx + (1.0f - d.blend) * d.I1x[o + k];
        iy[c] = d.blend * vy + (1.0f - d.blend) * d.I1y[o + k];
      }
    }
  } else {
    const bool out = (x2 > (float)W) || (x2 < 1.0f) || (y2 > (float)H) || (y2 < 1.0f) || !(x2 == x2) || !(y2 == y2);
    if (out) {
      for (int c = 0; c < d.nc; ++c) it[c] = ix[c] = iy[c] = 0.0f;
      return;
    }
    const float r = y2 - 1.0f, q = x2 - 1.0f;
    if (INTERP == OF_INTERP_CUBIC) {
      const int i0 = (int)floorf(r), j0 = (int)floorf(q);
      float wr[4], wc[4];
      int rr[4], cc[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        wr[a] = bspline3(r - (float)(i0 + a - 1));
        wc[a] = bspline3(q - (float)(j0 + a - 1));
        rr[a] = ext_mirror(i0 + a - 1, H);
        cc[a] = ext_mirror(j0 + a - 1, W);
      }
      for (int c = 0; c < d.nc; ++c) {
        const size_t o = c * ps;
        float v = 0.0f, vx = 0.0f, vy = 0.0f;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          float tv = 0.0f, tx = 0.0f, ty = 0.0f;
          const size_t rb = o + (size_t)rr[a] * P;
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            tv += wc[b] * d.Cc[rb + cc[b]];
            tx += wc[b] * d.A[rb + cc[b]];
            ty += wc[b] * d.B[rb + cc[b]];
          }
          v += wr[a] * tv;
          vx += wr[a] * tx;
          vy += wr[a] * ty;
        }
        it[c] = v - d.I1[o + k];
        ix[c] = d.blend * vx + (1.0f - d.blend) * d.I1x[o + k];
        iy[c] = d.blend * vy + (1.0f - d.blend) * d.I1y[o + k];
      }
    } else {  // bi-linear
      int i0 = (int)floorf(r), j0 = (int)floorf(q);
      float fr = r - i0, fc = q - j0;
      int i1 = min(i0 + 1, H - 1), j1 = min(j0 + 1, W - 1);
      for (int c = 0; c < d.nc; ++c) {
        const size_t o = c * ps;
        auto bil = [&](const float *p) {
          const float *r0 = p + o + (size_t)i0 * P, *r1 = p + o + (size_t)i1 * P;
          return (1.0f - fr) * ((1.0f - fc) * r0[j0] + fc * r0[j1]) + fr * ((1.0f - fc) * r1[j0] + fc * r1[j1]);
        };
        it[c] = bil(d.I2) - d.I1[o + k];
        ix[c] = d.blend * bil(d.A) + (1.0f - d.blend) * d.I1x[o + k];
        iy[c] = d.blend * bil(d.B) + (1.0f - d.blend) * d.I1y[o + k];
      }
    }
  }
}

#define OF_MAX_NC 4

template <int INTERP>
__global__ void k_partial_deriv(DerivArgs d, const float2 *__restrict__ uv, int H, int W, int P, size_t ps,
                                float *__restrict__ It, float *__restrict__ Ix, float *__restrict__ Iy) {
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    float2 f = uv[k];
    float it[OF_MAX_NC], ix[OF_MAX_NC], iy[OF_MAX_NC];
    warp_pixel<INTERP>(d, H, W, P, ps, i, j, (float)(j + 1) + f.x, (float)(i + 1) + f.y, it, ix, iy);
    for (int c = 0; c < d.nc; ++c) {
      It[c * ps + k] = it[c];
      Ix[c * ps + k] = ix[c];
      Iy[c * ps + k] = iy[c];
    }
  }
}
template __global__ void k_partial_deriv<0>(DerivArgs, const float2 *, int, int, int, size_t, float *, float *, float *);
template __global__ void k_partial_deriv<1>(DerivArgs, const float2 *, int, int, int, size_t, float *, float *, float *);
template __global__ void k_partial_deriv<2>(DerivArgs, const float2 *, int, int, int, size_t, float *, float *, float *);

// ---------------------------------------------------------------------------
// matrix-free flow operator
__device__ __forceinline__ float2 edge_w(const OpArgs &o, int axis, float du, float dv) {
  float wu = 0.0f, wv = 0.0f;
  if (o.use_q) { wu += o.aq_s * pen_w(o.qsu[axis], du); wv += o.aq_s * pen_w(o.qsv[axis], dv); }
  if (o.use_r) { wu += o.ar_s * pen_w(o.rsu[axis], du); wv += o.ar_s * pen_w(o.rsv[axis], dv); }
  return make_float2(wu, wv);
}

__device__ __forceinline__ float2 ld_uvd(const float2 *uv, const float2 *duv, size_t k) {
  float2 a = uv[k];
  if (duv) { float2 b = duv[k]; a.x += b.x; a.y += b.y; }
  return a;
}

// coef planes: 0 wx_u, 1 wy_u, 2 wx_v, 3 wy_v, 4 a_uu, 5 a_uv, 6 a_vv; rhs float2
__global__ void k_flow_operator(OpArgs o, const float2 *__restrict__ uv, const float2 *__restrict__ duv,
                                const float *__restrict__ It, const float *__restrict__ Ix, const float *__restrict__ Iy,
                                int nc, const float2 *__restrict__ uvhat, int H, int W, int P, size_t ps,
                                float *__restrict__ coef, float2 *__restrict__ rhs) {
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    const float2 c = ld_uvd(uv, duv, k);
    float2 eR = make_float2(0.f, 0.f), eD = eR, eL = eR, eU = eR;
    if (j < W - 1) { float2 n = ld_uvd(uv, duv, k + 1); eR = edge_w(o, 0, n.x - c.x, n.y - c.y); }
    if (i < H - 1) { float2 n = ld_uvd(uv, duv, k + P); eD = edge_w(o, 1, n.x - c.x, n.y - c.y); }
    if (j > 0) { float2 n = ld_uvd(uv, duv, k - 1); eL = edge_w(o, 0, c.x - n.x, c.y - n.y); }
    if (i > 0) { float2 n = ld_uvd(uv, duv, k - P); eU = edge_w(o, 1, c.x - n.x, c.y - n.y); }
    // data term, channel-averaged (classic_nl.py:330-343)
    float du = 0.f, dv = 0.f;
    if (duv) { du = duv[k].x; dv = duv[k].y; }
    float psq = 0.f, psr = 0.f, ix2 = 0.f, iy2 = 0.f, ixy = 0.f, itx = 0.f, ity = 0.f;
    for (int ch = 0; ch < nc; ++ch) {
      const size_t kc = ch * ps + k;
      const float gx = Ix[kc], gy = Iy[kc], itl = It[kc] + gx * du + gy * dv;
      if (o.use_q) psq += pen_w(o.qd, itl);
      if (o.use_r) psr += pen_w(o.rd, itl);
      ix2 += gx * gx; iy2 += gy * gy; ixy += gx * gy;
      itx += itl * gx; ity += itl * gy;
    }
    const float inv = 1.0f / (float)nc;
    const float psi = ((o.use_q ? o.aq_d * psq : 0.f) + (o.use_r ? o.ar_d * psr : 0.f)) * inv;
    ix2 *= inv; iy2 *= inv; ixy *= inv; itx *= inv; ity *= inv;
    // b uses uv (not uv + duv): classic_nl.py:362-367
    const float2 u0 = uv[k];
    float lu = 0.f, lv = 0.f;
    if (j < W - 1) { float2 n = uv[k + 1]; lu += eR.x * (u0.x - n.x); lv += eR.y * (u0.y - n.y); }
    if (i < H - 1) { float2 n = uv[k + P]; lu += eD.x * (u0.x - n.x); lv += eD.y * (u0.y - n.y); }
    if (j > 0) { float2 n = uv[k - 1]; lu += eL.x * (u0.x - n.x); lv += eL.y * (u0.y - n.y); }
    if (i > 0) { float2 n = uv[k - P]; lu += eU.x * (u0.x - n.x); lv += eU.y * (u0.y - n.y); }
    float auu = psi * ix2 + (eL.x + eR.x + eU.x + eD.x);
    float avv = psi * iy2 + (eL.y + eR.y + eU.y + eD.y);
    float bu = -lu - psi * itx, bv = -lv - psi * ity;
    if (uvhat) {  // AltBA coupling (alt_ba.py:236-242)
      const float2 h = uvhat[k];
      const float tu = pen_w(o.rc, u0.x - h.x), tv = pen_w(o.rc, u0.y - h.y);
      auu += o.lambda2 * tu;
      avv += o.lambda2 * tv;
      bu += o.lambda2 * tu * (h.x - u0.x);
      bv += o.lambda2 * tv * (h.y - u0.y);
    }
    coef[k] = eR.x;
    coef[ps + k] = eD.x;
    coef[2 * ps + k] = eR.y;
    coef[3 * ps + k] = eD.y;
    coef[4 * ps + k] = auu;
    coef[5 * ps + k] = psi * ixy;
    coef[6 * ps + k] = avv;
    rhs[k] = make_float2(bu, bv);
  }
}

// ---------------------------------------------------------------------------
// IRLS update: uv1 = uv + clip(x) (classic_nl.py:250-262); with occ != nullptr
// also detect_occlusion(uv1, images) (occlusion.py:6-56), where uv1 at the
// left / upper neighbour is recomputed in-register.
__device__ __forceinline__ float2 upd(const float2 *uv, const float2 *x, size_t k, int clip) {
  float2 a = uv[k], b = x[k];
  if (clip) { b.x = fminf(fmaxf(b.x, -1.0f), 1.0f); b.y = fminf(fmaxf(b.y, -1.0f), 1.0f); }
  return make_float2(a.x + b.x, a.y + b.y);
}

__global__ void k_update_occ(const float2 *__restrict__ uv, const float2 *__restrict__ x, int clip,
                             float2 *__restrict__ uv1, const float *__restrict__ I1, const float *__restrict__ I2,
                             int nc, float *__restrict__ occ, int H, int W, int P, size_t ps) {
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    const float2 c = upd(uv, x, k, clip);
    uv1[k] = c;
    if (!occ) continue;
    float dudx = j > 0 ? c.x - upd(uv, x, k - 1, clip).x : 0.0f;
    float dvdy = i > 0 ? c.y - upd(uv, x, k - P, clip).y : 0.0f;
    float div = dudx + dvdy;
    float odiv = expf(-div * div * (1.0f / (2.0f * 0.3f * 0.3f)));
    // bilinear warp of frame 2, 0-based, coordinates clamped ('nearest')
    float r = fminf(fmaxf((float)i + c.y, 0.0f), (float)(H - 1));
    float q = fminf(fmaxf((float)j + c.x, 0.0f), (float)(W - 1));
    int i0 = (int)floorf(r), j0 = (int)floorf(q);
    float fr = r - i0, fc = q - j0;
    int i1 = min(i0 + 1, H - 1), j1 = min(j0 + 1, W - 1);
    float it = 0.0f;
    for (int ch = 0; ch < nc; ++ch) {
      const float *b = I2 + ch * ps;
      const float *r0 = b + (size_t)i0 * P, *r1 = b + (size_t)i1 * P;
      float w = (1.0f - fr) * ((1.0f - fc) * r0[j0] + fc * r0[j1]) + fr * ((1.0f - fc) * r1[j0] + fc * r1[j1]);
      it += fabsf(w - I1[ch * ps + k]);
    }
    if (nc > 1) it /= (float)nc;
    occ[k] = odiv * expf(-it * it * (1.0f / (2.0f * 20.0f * 20.0f)));
  }
}

// in-place uv += x (HS, hs.py:130-134), optional clip
__global__ void k_add_update(float2 *__restrict__ uv, const float2 *__restrict__ x, int clip, int H, int W, int P) {
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    uv[k] = upd(uv, x, k, clip);
  }
}

// uv = uv + (b - a): the duv bookkeeping of classic_nl.py:271-275 / ba.py:404-407
__global__ void k_axpy_diff(float2 *__restrict__ uv, const float2 *__restrict__ a, const float2 *__restrict__ b, int H,
                            int W, int P) {
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    float2 u = uv[k], x = a[k], y = b[k];
    uv[k] = make_float2(u.x + (y.x - x.x), u.y + (y.y - x.y));
  }
}

// out = b - a
__global__ void k_sub2(const float2 *__restrict__ a, const float2 *__restrict__ b, float2 *__restrict__ out, int H,
                       int W, int P) {
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    float2 x = a[k], y = b[k];
    out[k] = make_float2(y.x - x.x, y.y - x.y);
  }
}

// ---------------------------------------------------------------------------
// scipy.ndimage.median_filter(size=S, mode='reflect'): rank selection with
// index tie-break (the element of rank S*S/2), branch-free.
template <int S>
__device__ __forceinline__ float median_window(const float *a) {
  constexpr int N = S * S;
  float m = a[0];
#pragma unroll
  for (int t = 0; t < N; ++t) {
    int cnt = 0;
#pragma unroll
    for (int u = 0; u < N; ++u) cnt += (a[u] < a[t]) || (a[u] == a[t] && u < t);
    m = cnt == N / 2 ? a[t] : m;
  }
  return m;
}

template <int S>
__global__ void k_median2(const float2 *__restrict__ in, float2 *__restrict__ out, int H, int W, int P) {
  constexpr int h = S / 2;
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    float au[S * S], av[S * S];
    int t = 0;
#pragma unroll
    for (int a = -h; a <= h; ++a) {
      const float2 *row = in + (size_t)ext_reflect(i + a, H) * P;
#pragma unroll
      for (int b = -h; b <= h; ++b, ++t) {
        float2 v = row[ext_reflect(j + b, W)];
        au[t] = v.x;
        av[t] = v.y;
      }
    }
    out[(size_t)i * P + j] = make_float2(median_window<S>(au), median_window<S>(av));
  }
}

template <int S>
__global__ void k_median1(const float *__restrict__ in, float *__restrict__ out, int H, int W, int P, size_t ps) {
  constexpr int h = S / 2;
  in += blockIdx.z * ps;
  out += blockIdx.z * ps;
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    float a[S * S];
    int t = 0;
#pragma unroll
    for (int y = -h; y <= h; ++y) {
      const float *row = in + (size_t)ext_reflect(i + y, H) * P;
#pragma unroll
      for (int x = -h; x <= h; ++x, ++t) a[t] = row[ext_reflect(j + x, W)];
    }
    out[(size_t)i * P + j] = median_window<S>(a);
  }
}
template __global__ void k_median2<3>(const float2 *, float2 *, int, int, int);
template __global__ void k_median2<5>(const float2 *, float2 *, int, int, int);
template __global__ void k_median2<7>(const float2 *, float2 *, int, int, int);
template __global__ void k_median1<3>(const float *, float *, int, int, int, size_t);
template __global__ void k_median1<5>(const float *, float *, int, int, int, size_t);
template __global__ void k_median1<7>(const float *, float *, int, int, int, size_t);

// uv_tilde = u + lam * (un - u) (denoise_LO, denoising.py:28-29)
__global__ void k_lo_blend(const float2 *__restrict__ u, const float2 *__restrict__ un, float lam,
                           float2 *__restrict__ out, int H, int W, int P) {
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    float2 a = u[k], b = un[k];
    out[k] = make_float2(a.x + lam * (b.x - a.x), a.y + lam * (b.y - a.y));
  }
}

// ---------------------------------------------------------------------------
// Occlusion-weighted, colour-guided weighted median
// (denoise_color_weighted_medfilt2, weighted_median.py:24-112).  One wave per 8x8 tile:
//  1. the (8+2h)^2 region is loaded straight into registers, NPER keys per
//     lane (element e = lane*NPER + r), and guide+occ records go to LDS;
//  2. u and v keys are bitonic-sorted in registers: stages with partner
//     distance < NPER swap registers, the others exchange with lane^(d/NPER)
//     by ds_bpermute (no LDS storage, no barriers);
//  3. sorted keys go to LDS; every lane walks both lists in lockstep, 8 keys
//     per batch, weights of the u and v samples computed in packed fp32
//     (v_pk_*), fp64 cumulative sums advanced branch-free in sorted order.
// Weight = max(2^(-|dlab|^2 * log2e/(2 sigma^2)) * occ, 1e-10) (v_exp_f32);
// result = the first sorted value with cumsum >= total/2
// (weighted_median.py:5-21, :67-112).
#define WMF_T 8
template <int GC>
struct WmfRec;
template <>
struct WmfRec<3> {
  using T = float4;
  __device__ static T make(float a, float b, float c, float o) { return make_float4(a, b, c, o); }
  __device__ static float d2(const T &s, const float *cg) {
    const float e0 = s.x - cg[0], e1 = s.y - cg[1], e2 = s.z - cg[2];
    return e0 * e0 + e1 * e1 + e2 * e2;
  }
  __device__ static float occ(const T &s) { return s.w; }
};
template <>
struct WmfRec<1> {
  using T = float2;
  __device__ static T make(float a, float, float, float o) { return make_float2(a, o); }
  __device__ static float d2(const T &s, const float *cg) {
    const float e0 = s.x - cg[0];
    return e0 * e0;
  }
  __device__ static float occ(const T &s) { return s.y; }
};

typedef float wmf_v2f __attribute__((ext_vector_type(2)));

// weight of region sample s for a pixel of guide colour (c01, c2):
// max(2^(nk |dlab|^2) occ, 1e-10), channels 0-1 in packed fp32
__device__ __forceinline__ float wmf_w(const float4 &s, wmf_v2f c01, float c2, float nk) {
  const wmf_v2f e = wmf_v2f{s.x, s.y} - c01, q = e * e;
  const float e2 = s.z - c2;
  return fmaxf(__builtin_amdgcn_exp2f(fmaf(e2, e2, q.x + q.y) * nk) * s.w, 1e-10f);
}
__device__ __forceinline__ float wmf_w(const float2 &s, wmf_v2f c01, float, float nk) {
  const float e = s.x - c01.x;
  return fmaxf(__builtin_amdgcn_exp2f(e * e * nk) * s.y, 1e-10f);
}

template <int NPER>
__device__ __forceinline__ void bitonic_regs(uint64_t (&k)[NPER], int lane) {
  constexpr int N = NPER * 64;
#pragma unroll
  for (int kk = 2; kk <= N; kk <<= 1) {
#pragma unroll
    for (int jj = kk >> 1; jj > 0; jj >>= 1) {
      if (jj >= NPER) {
        const int lj = jj / NPER;
        const bool lower = (lane & lj) == 0;
#pragma unroll
        for (int r = 0; r < NPER; ++r) {
          const bool up = (((lane * NPER + r) & kk) == 0);
          const uint64_t o = __shfl_xor(k[r], lj);
          const bool take_min = lower == up;
          const uint64_t mn = k[r] < o ? k[r] : o, mx = k[r] < o ? o : k[r];
          k[r] = take_min ? mn : mx;
        }
      } else {
#pragma unroll
        for (int r = 0; r < NPER; ++r) {
          const int rp = r ^ jj;
          if (rp > r) {
            const bool up = (((lane * NPER + r) & kk) == 0);
            const uint64_t a = k[r], b = k[rp];
            const bool sw = (a > b) == up;
            k[r] = sw ? b : a;
            k[rp] = sw ? a : b;
          }
        }
      }
    }
  }
}

template <int GC, int NPER>
__global__ __launch_bounds__(64) void k_wmf(const float2 *__restrict__ uv, const float *__restrict__ guide,
                                             const float *__restrict__ occ, float2 *__restrict__ out, int H, int W,
                                             int P, size_t ps, int hsz, float nk, int RW, int nreg) {
  using R = WmfRec<GC>;
  using T = typename R::T;
  constexpr int N = NPER * 64;
  // LDS: sorted region positions (ry << 8 | rx) of the u and v lists, then
  // the guide+occ records: 2*N*2 + nreg*sizeof(T) bytes (9.8 KB at h = 7)
  extern __shared__ uint64_t lds_u64[];
  T *smp = reinterpret_cast<T *>(lds_u64);  // [nreg]
  uint16_t *ku = reinterpret_cast<uint16_t *>(smp + nreg), *kv = ku + N;
  const int ty0 = blockIdx.y * WMF_T, tx0 = blockIdx.x * WMF_T;
  const int lane = threadIdx.x;
  uint64_t a[NPER], b[NPER];
#pragma unroll
  for (int r = 0; r < NPER; ++r) {
    const int s = lane * NPER + r;
    a[r] = ~0ull;
    b[r] = ~0ull;
    if (s < nreg) {
      const int ry = s / RW, rx = s - ry * RW;
      const size_t g = (size_t)ext_mirror(ty0 - hsz + ry, H) * P + ext_mirror(tx0 - hsz + rx, W);
      const float2 v = uv[g];
      const uint64_t lo = ((uint64_t)ry << 8) | (uint64_t)rx;
      a[r] = ((uint64_t)f2ord(v.x) << 32) | lo;
      b[r] = ((uint64_t)f2ord(v.y) << 32) | lo;
      float gv[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < GC; ++c) gv[c] = guide[c * ps + g];
      smp[s] = R::make(gv[0], gv[1], gv[2], occ[g]);
    }
  }
  bitonic_regs<NPER>(a, lane);
  bitonic_regs<NPER>(b, lane);
#pragma unroll
  for (int r = 0; r < NPER; ++r) {
    ku[lane * NPER + r] = (uint16_t)a[r];  // padding keys -> 0xffff: out of every window
    kv[lane * NPER + r] = (uint16_t)b[r];
  }
  __syncthreads();
  const int py = lane >> 3, px = lane & 7;
  const int gi = ty0 + py, gj = tx0 + px;
  const bool live = gi < H && gj < W;  // dead lanes still walk (wave-uniform exit)
  float cg[3] = {0.f, 0.f, 0.f};
  {
    const T c0 = smp[(py + hsz) * RW + px + hsz];
    const float *cf = reinterpret_cast<const float *>(&c0);
#pragma unroll
    for (int c = 0; c < GC; ++c) cg[c] = cf[c];
  }
  const wmf_v2f c01 = {cg[0], cg[1]};
  // total weight of the lane's window (row-major window order)
  double tot = 0.0;
  for (int dy = 0; dy <= 2 * hsz; ++dy) {
    const T *row = smp + (py + dy) * RW + px;
    for (int dx = 0; dx <= 2 * hsz; ++dx) tot += (double)wmf_w(row[dx], c01, cg[2], nk);
  }
  const double half = 0.5 * tot;
  const unsigned span = 2u * hsz;
  double cu = 0.0, cv = 0.0;
  unsigned resu = 0, resv = 0;
  bool du = !live, dv = !live;
  for (int k0 = 0; k0 < N; k0 += 8) {
    // keys are wave-uniform: each sample record is one broadcast LDS read,
    // the per-lane part is the window test
    unsigned ka[8], kb[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      ka[i] = ku[k0 + i];
      kb[i] = kv[k0 + i];
    }
    float wa[8], wb[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const unsigned rya = ka[i] >> 8, rxa = ka[i] & 0xffu, ryb = kb[i] >> 8, rxb = kb[i] & 0xffu;
      const bool ina = (rya - (unsigned)py) <= span && (rxa - (unsigned)px) <= span;
      const bool inb = (ryb - (unsigned)py) <= span && (rxb - (unsigned)px) <= span;
      // padding keys (0xffff) are outside every window; read any record
      const float xa = wmf_w(smp[ka[i] == 0xffffu ? 0u : rya * RW + rxa], c01, cg[2], nk);
      const float xb = wmf_w(smp[kb[i] == 0xffffu ? 0u : ryb * RW + rxb], c01, cg[2], nk);
      wa[i] = ina ? xa : 0.0f;
      wb[i] = inb ? xb : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      cu += (double)wa[i];
      cv += (double)wb[i];
      const bool xa = !du && cu >= half, xb = !dv && cv >= half;
      resu = xa ? ka[i] : resu;
      resv = xb ? kb[i] : resv;
      du = du || xa;
      dv = dv || xb;
    }
    if (__all(du && dv)) break;
  }
  if (live) {
    // the selected samples' values, re-read at their (mirrored) positions
    const int ya = ext_mirror(ty0 - hsz + (int)(resu >> 8), H), xa = ext_mirror(tx0 - hsz + (int)(resu & 0xffu), W);
    const int yb = ext_mirror(ty0 - hsz + (int)(resv >> 8), H), xb = ext_mirror(tx0 - hsz + (int)(resv & 0xffu), W);
    out[(size_t)gi * P + gj] = make_float2(uv[(size_t)ya * P + xa].x, uv[(size_t)yb * P + xb].y);
  }
}
#define OF_WMF(GC, NP)                                                                                           \
  template __global__ void k_wmf<GC, NP>(const float2 *, const float *, const float *, float2 *, int, int, int, \
                                          size_t, int, float, int, int);
OF_WMF(1, 1) OF_WMF(1, 2) OF_WMF(1, 4) OF_WMF(1, 8) OF_WMF(1, 16)
OF_WMF(3, 1) OF_WMF(3, 2) OF_WMF(3, 4) OF_WMF(3, 8) OF_WMF(3, 16)
#undef OF_WMF
