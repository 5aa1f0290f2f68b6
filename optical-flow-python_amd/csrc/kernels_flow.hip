// kernels_flow.hip — the per-warping-iteration kernels of the IRLS loop:
// warp + derivatives, matrix-free flow-operator assembly, update/clip +
// occlusion, 5x5 median and the occlusion-weighted colour-guided weighted
// median.  See DESIGN.md for the roofline of each.
#include "kernels.h"

// ---------------------------------------------------------------------------
// cubic Hermite basis (tensor-product form of derivatives.py:7-24's
// 16x16 bicubic coefficient matrix)
__device__ __forceinline__ void hermite(float t, float h[4], float dh[4]) {
  OF_NOCONTRACT
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
  OF_NOCONTRACT
  t = fabsf(t);
  if (t < 1.0f) return 2.0f / 3.0f - t * t + 0.5f * t * t * t;
  if (t < 2.0f) {
    float s = 2.0f - t;
    return s * s * s * (1.0f / 6.0f);
  }
  return 0.0f;
}

// partial_deriv (derivatives.py:148-296) for one pixel and all channels.
// (x2, y2) are the 1-based warped coordinates.  Each channel's (It, Ix, Iy)
// goes to out(c, it, ix, iy): PlaneOut stores it straight to the planes (no
// per-channel register arrays: a runtime-indexed array would live in
// scratch); RegOut<NC> keeps it in registers for the fused warp + assembly
// (NC > 0: the channel loop is unrolled, so the array index is static).
struct PlaneOut {
  float *It, *Ix, *Iy;
  size_t ps, k;
  __device__ __forceinline__ void operator()(int c, float it, float ix, float iy) const {
    It[c * ps + k] = it;
    Ix[c * ps + k] = ix;
    Iy[c * ps + k] = iy;
  }
};
template <int NC>
struct RegOut {
  float it[NC], ix[NC], iy[NC];
  __device__ __forceinline__ void operator()(int c, float a, float b, float e) {
    it[c] = a;
    ix[c] = b;
    iy[c] = e;
  }
};
template <int INTERP, int NC, typename Out>
__device__ __forceinline__ void warp_pixel(const DerivArgs &d, int H, int W, int P, size_t ps, int i, int j, float x2,
                                           float y2, Out &out) {
  OF_NOCONTRACT
  const size_t k = (size_t)i * P + j;
  const int nc = NC > 0 ? NC : d.nc;
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
#pragma unroll
    for (int c = 0; c < nc; ++c) {
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
      if (oob) out(c, 0.0f, 0.0f, 0.0f);
      else
        out(c, v - d.I1[o + k], d.blend * vx + (1.0f - d.blend) * d.I1x[o + k],
            d.blend * vy + (1.0f - d.blend) * d.I1y[o + k]);
    }
  } else {
    const bool outside = (x2 > (float)W) || (x2 < 1.0f) || (y2 > (float)H) || (y2 < 1.0f) || !(x2 == x2) || !(y2 == y2);
    if (outside) {
#pragma unroll
      for (int c = 0; c < nc; ++c) out(c, 0.0f, 0.0f, 0.0f);
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
#pragma unroll
      for (int c = 0; c < nc; ++c) {
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
        out(c, v - d.I1[o + k], d.blend * vx + (1.0f - d.blend) * d.I1x[o + k],
            d.blend * vy + (1.0f - d.blend) * d.I1y[o + k]);
      }
    } else {  // bi-linear
      int i0 = (int)floorf(r), j0 = (int)floorf(q);
      float fr = r - i0, fc = q - j0;
      int i1 = min(i0 + 1, H - 1), j1 = min(j0 + 1, W - 1);
#pragma unroll
      for (int c = 0; c < nc; ++c) {
        const size_t o = c * ps;
        auto bil = [&](const float *p) {
          const float *r0 = p + o + (size_t)i0 * P, *r1 = p + o + (size_t)i1 * P;
          return (1.0f - fr) * ((1.0f - fc) * r0[j0] + fc * r0[j1]) + fr * ((1.0f - fc) * r1[j0] + fc * r1[j1]);
        };
        out(c, bil(d.I2) - d.I1[o + k], d.blend * bil(d.A) + (1.0f - d.blend) * d.I1x[o + k],
            d.blend * bil(d.B) + (1.0f - d.blend) * d.I1y[o + k]);
      }
    }
  }
}


// launch bounds = the grid2 block (64 x 4): without them the compiler
// assumes 1024-thread blocks, caps VGPRs at 128 and spills to scratch
template <int INTERP>
__global__ __launch_bounds__(OF_BX *OF_BY) void k_partial_deriv(DerivArgs d, const float2 *__restrict__ uv, int H,
                                                                int W, int P, size_t ps, float *__restrict__ It,
                                                                float *__restrict__ Ix, float *__restrict__ Iy) {
  OF_FOR_PIXELS_XCD(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    float2 f = uv[k];
    PlaneOut out{It, Ix, Iy, ps, k};
    warp_pixel<INTERP, 0>(d, H, W, P, ps, i, j, (float)(j + 1) + f.x, (float)(i + 1) + f.y, out);
  }
}
template __global__ void k_partial_deriv<0>(DerivArgs, const float2 *, int, int, int, size_t, float *, float *, float *);
template __global__ void k_partial_deriv<1>(DerivArgs, const float2 *, int, int, int, size_t, float *, float *, float *);
template __global__ void k_partial_deriv<2>(DerivArgs, const float2 *, int, int, int, size_t, float *, float *, float *);

// ---------------------------------------------------------------------------
// matrix-free flow operator
// Penalty mode of an assembly kernel: OF_PM_ANY decides everything at run
// time (use_q / use_r, each penalty's kind); otherwise the system is the
// quadratic relaxation only (OF_PM_Q, alpha == 1, every penalty quadratic) or
// the robust one only (OF_PM_R(kind), alpha == 0, every robust penalty of
// that kind).  The arithmetic is the generic form's, term for term.
#define OF_PM_ANY (-1)
#define OF_PM_Q 0
#define OF_PM_R(kind) (1 + (kind))
template <int M>
struct PenMode {
  static constexpr bool any = M == OF_PM_ANY;
  static constexpr int kind = M == OF_PM_ANY ? -1 : M == OF_PM_Q ? OF_PEN_QUADRATIC : M - 1;
  __device__ static bool q(const OpArgs &o) { return any ? o.use_q : M == OF_PM_Q; }
  __device__ static bool r(const OpArgs &o) { return any ? o.use_r : M != OF_PM_Q; }
  __device__ static float pen(const PenF &p, float x) { return pen_k<kind>(p, x); }
};

template <int M = OF_PM_ANY>
__device__ __forceinline__ float2 edge_w(const OpArgs &o, int axis, float du, float dv) {
  OF_NOCONTRACT
  using PM = PenMode<M>;
  float wu = 0.0f, wv = 0.0f;
  if (PM::q(o)) { wu += o.aq_s * PM::pen(o.qsu[axis], du); wv += o.aq_s * PM::pen(o.qsv[axis], dv); }
  if (PM::r(o)) { wu += o.ar_s * PM::pen(o.rsu[axis], du); wv += o.ar_s * PM::pen(o.rsv[axis], dv); }
  return make_float2(wu, wv);
}

__device__ __forceinline__ float2 ld_uvd(const float2 *uv, const float2 *duv, size_t k) {
  float2 a = uv[k];
  if (duv) { float2 b = duv[k]; a.x += b.x; a.y += b.y; }
  return a;
}

// The flow at a pixel and its four neighbours, loaded together at clamped
// indices (a neighbour outside the image reads the pixel itself; its value
// is never used) and pinned in registers right away: loaded under the
// boundary branches, each load was a masked load waited for on its own --
// four more memory round trips per pixel row of the fused warp + assembly,
// after the gather's.
struct UvNbr {
  float2 c, r, d, l, u;
};
__device__ __forceinline__ UvNbr ld_nbr(const float2 *__restrict__ uv, int i, int j, int H, int W, int P) {
  const size_t k = (size_t)i * P + j;
  UvNbr n;
  n.c = uv[k];
  n.r = uv[j < W - 1 ? k + 1 : k];
  n.d = uv[i < H - 1 ? k + P : k];
  n.l = uv[j > 0 ? k - 1 : k];
  n.u = uv[i > 0 ? k - P : k];
  asm volatile("" : "+v"(n.c.x), "+v"(n.c.y), "+v"(n.r.x), "+v"(n.r.y), "+v"(n.d.x), "+v"(n.d.y), "+v"(n.l.x),
               "+v"(n.l.y), "+v"(n.u.x), "+v"(n.u.y));
  return n;
}

// coef planes: 0 wx_u, 1 wy_u, 2 wx_v, 3 wy_v, 4 a_uu, 5 a_uv, 6 a_vv; rhs float2.
// One pixel's row of the system; deriv(ch, It, Ix, Iy) fetches channel ch's
// derivatives (planes, or the fused kernel's registers).  nb: the flow of
// the pixel and its neighbours already in registers (ld_nbr; only without
// duv), else loaded here.
template <int NC, int M, typename Deriv>
__device__ __forceinline__ void assemble_px(const OpArgs &o, const float2 *__restrict__ uv,
                                            const float2 *__restrict__ duv, int nc_rt, const float2 *__restrict__ uvhat,
                                            int i, int j, int H, int W, int P, size_t ps, float *__restrict__ coef,
                                            float2 *__restrict__ rhs, const Deriv &deriv, const UvNbr *nb = nullptr) {
  OF_NOCONTRACT
  using PM = PenMode<M>;
  const int nc = NC > 0 ? NC : nc_rt;
  const size_t k = (size_t)i * P + j;
  const float2 c = nb ? nb->c : ld_uvd(uv, duv, k);
  float2 eR = make_float2(0.f, 0.f), eD = eR, eL = eR, eU = eR;
  if (j < W - 1) { float2 n = nb ? nb->r : ld_uvd(uv, duv, k + 1); eR = edge_w<M>(o, 0, n.x - c.x, n.y - c.y); }
  if (i < H - 1) { float2 n = nb ? nb->d : ld_uvd(uv, duv, k + P); eD = edge_w<M>(o, 1, n.x - c.x, n.y - c.y); }
  if (j > 0) { float2 n = nb ? nb->l : ld_uvd(uv, duv, k - 1); eL = edge_w<M>(o, 0, c.x - n.x, c.y - n.y); }
  if (i > 0) { float2 n = nb ? nb->u : ld_uvd(uv, duv, k - P); eU = edge_w<M>(o, 1, c.x - n.x, c.y - n.y); }
  // data term, channel-averaged (classic_nl.py:330-343)
  float du = 0.f, dv = 0.f;
  if (duv) { du = duv[k].x; dv = duv[k].y; }
  float psq = 0.f, psr = 0.f, ix2 = 0.f, iy2 = 0.f, ixy = 0.f, itx = 0.f, ity = 0.f;
#pragma unroll
  for (int ch = 0; ch < nc; ++ch) {
    float it, gx, gy;
    deriv(ch, it, gx, gy);
    const float itl = it + gx * du + gy * dv;
    if (PM::q(o)) psq += PM::pen(o.qd, itl);
    if (PM::r(o)) psr += PM::pen(o.rd, itl);
    ix2 += gx * gx; iy2 += gy * gy; ixy += gx * gy;
    itx += itl * gx; ity += itl * gy;
  }
  const float inv = 1.0f / (float)nc;
  const float psi = ((PM::q(o) ? o.aq_d * psq : 0.f) + (PM::r(o) ? o.ar_d * psr : 0.f)) * inv;
  ix2 *= inv; iy2 *= inv; ixy *= inv; itx *= inv; ity *= inv;
  // b uses uv (not uv + duv): classic_nl.py:362-367
  const float2 u0 = nb ? nb->c : uv[k];
  float lu = 0.f, lv = 0.f;
  if (j < W - 1) { float2 n = nb ? nb->r : uv[k + 1]; lu += eR.x * (u0.x - n.x); lv += eR.y * (u0.y - n.y); }
  if (i < H - 1) { float2 n = nb ? nb->d : uv[k + P]; lu += eD.x * (u0.x - n.x); lv += eD.y * (u0.y - n.y); }
  if (j > 0) { float2 n = nb ? nb->l : uv[k - 1]; lu += eL.x * (u0.x - n.x); lv += eL.y * (u0.y - n.y); }
  if (i > 0) { float2 n = nb ? nb->u : uv[k - P]; lu += eU.x * (u0.x - n.x); lv += eU.y * (u0.y - n.y); }
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

template <int M>
__global__ __launch_bounds__(OF_BX *OF_BY) void k_flow_operator(OpArgs o, const float2 *__restrict__ uv, const float2 *__restrict__ duv,
                                const float *__restrict__ It, const float *__restrict__ Ix, const float *__restrict__ Iy,
                                int nc, const float2 *__restrict__ uvhat, int H, int W, int P, size_t ps,
                                float *__restrict__ coef, float2 *__restrict__ rhs) {
  OF_FOR_PIXELS_XCD(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    assemble_px<0, M>(o, uv, duv, nc, uvhat, i, j, H, W, P, ps, coef, rhs, [&](int ch, float &it, float &gx, float &gy) {
      const size_t kc = ch * ps + k;
      it = It[kc];
      gx = Ix[kc];
      gy = Iy[kc];
    });
  }
}

// Warp + derivatives + assembly in one pass: the
// per-channel It / Ix / Iy of a pixel stay in registers, so the 24 B/px
// round trip of the three planes (nc = 1) and one launch per warping
// iteration go away.  The same arithmetic as k_partial_deriv +
// k_flow_operator, bitwise: no fma contraction in either (OF_WARP_NOCONTRACT;
// tests/test_gpu_stages.py).
template <int INTERP, int NC, int M>
__global__ __launch_bounds__(OF_BX *OF_BY) void k_warp_operator(DerivArgs d, OpArgs o, const float2 *__restrict__ uv,
                                                                int H, int W, int P, size_t ps,
                                                                float *__restrict__ coef, float2 *__restrict__ rhs) {
  OF_FOR_PIXELS_XCD(H, W) {
    if (j >= W) continue;
    // the pixel's and its neighbours' flow in one round trip, before the
    // gather that needs the pixel's
    const UvNbr nb = ld_nbr(uv, i, j, H, W, P);
    const float2 f = nb.c;
    RegOut<NC> r;
    warp_pixel<INTERP, NC>(d, H, W, P, ps, i, j, (float)(j + 1) + f.x, (float)(i + 1) + f.y, r);
    assemble_px<NC, M>(o, uv, (const float2 *)nullptr, NC, (const float2 *)nullptr, i, j, H, W, P, ps, coef, rhs,
                    [&](int ch, float &it, float &gx, float &gy) {
                      it = r.it[ch];
                      gx = r.ix[ch];
                      gy = r.iy[ch];
                    }, &nb);
  }
}
#define OF_WOP(I, N, M) template __global__ void k_warp_operator<I, N, M>(DerivArgs, OpArgs, const float2 *, int, int, \
                                                                          int, size_t, float *, float2 *);
#define OF_FOP(M) template __global__ void k_flow_operator<M>(OpArgs, const float2 *, const float2 *, const float *, \
                                                              const float *, const float *, int, const float2 *, int, \
                                                              int, int, size_t, float *, float2 *);
// specialised penalty modes: the registry's quadratic stage and its robust
// stages (generalized Charbonnier: Classic+NL; Charbonnier: Classic-C;
// Lorentzian: BA; Horn-Schunck's constant weights)
#define OF_PM_LIST(X) X(OF_PM_ANY) X(OF_PM_Q) X(OF_PM_R(OF_PEN_GEN_CHARBONNIER)) X(OF_PM_R(OF_PEN_CHARBONNIER)) \
  X(OF_PM_R(OF_PEN_LORENTZIAN)) X(OF_PM_R(OF_PEN_CONST))
#define OF_WOP_M(M) OF_WOP(0, 1, M) OF_WOP(1, 1, M) OF_WOP(2, 1, M) OF_WOP(0, 3, M) OF_WOP(1, 3, M) OF_WOP(2, 3, M)
OF_PM_LIST(OF_WOP_M)
OF_PM_LIST(OF_FOP)
#undef OF_WOP_M
#undef OF_WOP
#undef OF_FOP

// The same assembly with every intermediate in fp64 (the reference's own
// precision) and one rounding per stored plane: for AltBA (OpArgs::f64),
// whose robust systems are so ill-conditioned that the ~2e-7 relative error
// of the fp32 assembly's diagonal (a sum of four edge weights, a data term
// and the coupling) moved the solve by 5x the float32 floor of the system
// (tools/altba_gpu_probe.py).  Not on the hot path.
__device__ __forceinline__ double2 edge_w_f64(const OpArgs &o, int axis, double du, double dv) {
  double wu = 0.0, wv = 0.0;
  if (o.use_q) { wu += o.aq_s_d * pen_w_f64(o.qsu[axis], du); wv += o.aq_s_d * pen_w_f64(o.qsv[axis], dv); }
  if (o.use_r) { wu += o.ar_s_d * pen_w_f64(o.rsu[axis], du); wv += o.ar_s_d * pen_w_f64(o.rsv[axis], dv); }
  return make_double2(wu, wv);
}
__device__ __forceinline__ double2 ld_uvd_f64(const float2 *uv, const float2 *duv, size_t k) {
  const float2 a = uv[k];
  double2 r = make_double2(a.x, a.y);
  if (duv) { const float2 b = duv[k]; r.x += b.x; r.y += b.y; }
  return r;
}
__global__ __launch_bounds__(OF_BX *OF_BY) void k_flow_operator_f64(OpArgs o, const float2 *__restrict__ uv,
                                const float2 *__restrict__ duv, const float *__restrict__ It,
                                const float *__restrict__ Ix, const float *__restrict__ Iy, int nc,
                                const float2 *__restrict__ uvhat, int H, int W, int P, size_t ps,
                                float *__restrict__ coef, float2 *__restrict__ rhs) {
  OF_FOR_PIXELS_XCD(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    const double2 c = ld_uvd_f64(uv, duv, k);
    double2 eR = make_double2(0.0, 0.0), eD = eR, eL = eR, eU = eR;
    if (j < W - 1) { double2 n = ld_uvd_f64(uv, duv, k + 1); eR = edge_w_f64(o, 0, n.x - c.x, n.y - c.y); }
    if (i < H - 1) { double2 n = ld_uvd_f64(uv, duv, k + P); eD = edge_w_f64(o, 1, n.x - c.x, n.y - c.y); }
    if (j > 0) { double2 n = ld_uvd_f64(uv, duv, k - 1); eL = edge_w_f64(o, 0, c.x - n.x, c.y - n.y); }
    if (i > 0) { double2 n = ld_uvd_f64(uv, duv, k - P); eU = edge_w_f64(o, 1, c.x - n.x, c.y - n.y); }
    double du = 0.0, dv = 0.0;
    if (duv) { du = duv[k].x; dv = duv[k].y; }
    double psq = 0.0, psr = 0.0, ix2 = 0.0, iy2 = 0.0, ixy = 0.0, itx = 0.0, ity = 0.0;
    for (int ch = 0; ch < nc; ++ch) {
      const size_t kc = ch * ps + k;
      const double gx = Ix[kc], gy = Iy[kc], itl = It[kc] + gx * du + gy * dv;
      if (o.use_q) psq += pen_w_f64(o.qd, itl);
      if (o.use_r) psr += pen_w_f64(o.rd, itl);
      ix2 += gx * gx; iy2 += gy * gy; ixy += gx * gy;
      itx += itl * gx; ity += itl * gy;
    }
    const double inv = 1.0 / (double)nc;
    const double psi = ((o.use_q ? o.aq_d_d * psq : 0.0) + (o.use_r ? o.ar_d_d * psr : 0.0)) * inv;
    ix2 *= inv; iy2 *= inv; ixy *= inv; itx *= inv; ity *= inv;
    const float2 u0f = uv[k];
    const double2 u0 = make_double2(u0f.x, u0f.y);
    double lu = 0.0, lv = 0.0;
    if (j < W - 1) { float2 n = uv[k + 1]; lu += eR.x * (u0.x - n.x); lv += eR.y * (u0.y - n.y); }
    if (i < H - 1) { float2 n = uv[k + P]; lu += eD.x * (u0.x - n.x); lv += eD.y * (u0.y - n.y); }
    if (j > 0) { float2 n = uv[k - 1]; lu += eL.x * (u0.x - n.x); lv += eL.y * (u0.y - n.y); }
    if (i > 0) { float2 n = uv[k - P]; lu += eU.x * (u0.x - n.x); lv += eU.y * (u0.y - n.y); }
    double auu = psi * ix2 + (eL.x + eR.x + eU.x + eD.x);
    double avv = psi * iy2 + (eL.y + eR.y + eU.y + eD.y);
    double bu = -lu - psi * itx, bv = -lv - psi * ity;
    if (uvhat) {  // AltBA coupling (alt_ba.py:236-242)
      const float2 h = uvhat[k];
      const double tu = pen_w_f64(o.rc, u0.x - h.x), tv = pen_w_f64(o.rc, u0.y - h.y);
      auu += o.lambda2_d * tu;
      avv += o.lambda2_d * tv;
      bu += o.lambda2_d * tu * (h.x - u0.x);
      bv += o.lambda2_d * tv * (h.y - u0.y);
    }
    coef[k] = (float)eR.x;
    coef[ps + k] = (float)eD.x;
    coef[2 * ps + k] = (float)eR.y;
    coef[3 * ps + k] = (float)eD.y;
    coef[4 * ps + k] = (float)auu;
    coef[5 * ps + k] = (float)(psi * ixy);
    coef[6 * ps + k] = (float)avv;
    rhs[k] = make_float2((float)bu, (float)bv);
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
  OF_FOR_PIXELS_XCD(H, W) {
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
__global__ __launch_bounds__(OF_BX *OF_BY) void k_median2(const float2 *__restrict__ in, float2 *__restrict__ out, int H, int W, int P) {
  constexpr int h = S / 2;
  OF_FOR_PIXELS_XCD(H, W) {
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
__global__ __launch_bounds__(OF_BX *OF_BY) void k_median1(const float *__restrict__ in, float *__restrict__ out, int H, int W, int P, size_t ps) {
  constexpr int h = S / 2;
  in += blockIdx.z * ps;
  out += blockIdx.z * ps;
  OF_FOR_PIXELS_XCD(H, W) {
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
//  2. u and v keys (the value widened to fp64 with the region position in
//     its low mantissa bits, wmf_key) are bitonic-sorted in registers; each sample's sorted index e gives it a
//     chunk id e / CH (WMF_NC chunks of CH consecutive sorted samples per list);
//  3. every lane visits its own 15x15 window once (no out-of-window work):
//     weight w is added to the lane's chunk sums of the u and v lists
//     (ds_add_f64 into lane-private LDS slots, program order ->
//     deterministic); the window total is the sum of the chunk sums;
//  4. the chunk holding the half-weight crossing is found from the chunk
//     prefix sums; only that chunk's CH sorted samples are walked (per-lane
//     addresses) to the first one whose cumulative weight reaches total/2.
// LDS per wave at h = 7: 8 KB chunk sums + 8.4 KB records + 2 KB sorted
// positions + 1 KB chunk ids = 19.3 KB -> 8 waves per CU.
// Weight = max(2^(-|dlab|^2 * log2e/(2 sigma^2)) * occ, 1e-10) (v_exp_f32);
// result = the first sorted value with cumsum >= total/2
// (weighted_median.py:5-21, :67-112): the cumulative sum at a sorted sample
// is (chunk prefix) + (in-window weights before it in the chunk), the same
// sums the reference forms, summed in another order.
#define OF_MAX_NC 4  // image channels per frame the host accepts
#define WMF_T 8
#ifdef WMF_PHASE_TIMING  // tools/micro/wmf_phases.hip: per-wave phase timestamps
extern __device__ unsigned long long g_wmf_t[];
#define WMF_STAMP(i) \
  if (threadIdx.x == 0) g_wmf_t[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = clock64()
#else
#define WMF_STAMP(i)
#endif
#define WMF_NC 8
// (measured round 6 and removed: 16 chunks for the large regions, 0.888 vs
// 0.691 ms per 1080p launch at 5 instead of 8 waves per CU; a register
// accumulator per row for the middle sample's chunk, 0.828 vs 0.692 ms --
// DESIGN.md "Round 6 in brief" item 4)
__host__ __device__ constexpr int wmf_nc(int) { return WMF_NC; }
// WMF_WALK_LAST: the crossing sample found as the last one whose preceding
// sum is below half (1) or the first whose sum reaches half (0); the same
// sample either way (see the walk)
#ifndef WMF_WALK_LAST
#define WMF_WALK_LAST 1
#endif
// WMF_CID_PAIR: the u- and v-list chunk ids of a region sample side by side
// ([RW][RP][2] u8, one u16 read per window sample) instead of two planes
// ([2][RW][RP] u8, two u8 reads)
#ifndef WMF_CID_PAIR
#define WMF_CID_PAIR 0
#endif
// chunk-sum type: fp64 (default, 100 % exact on every fixture) or fp32
// (WMF_F32SUM: half the chunk-sum LDS).  The fp32 build emits native
// ds_add_f32 (checked in the ISA, no CAS loop) and yet runs 4.93 vs 0.83 ms
// per 1080p launch (99.996 % exact at h = 12; profiles/r3ac_wmf_f32sum.log):
// on gfx950 the fp32 LDS add is far slower than ds_add_f64 here.  Off.
#ifndef WMF_F32SUM
#define WMF_F32SUM 0
#endif
#if WMF_F32SUM
typedef float wmf_sum_t;
#define WMF_SUM_SHIFT 8
#else
typedef double wmf_sum_t;
#define WMF_SUM_SHIFT 9
#endif
template <int GC>
struct WmfRec;
template <>
struct WmfRec<3> {
  using T = float4;
  __device__ static T make(float a, float b, float c, float o) { return make_float4(a, b, c, o); }
};
template <>
struct WmfRec<1> {
  using T = float2;
  __device__ static T make(float a, float, float, float o) { return make_float2(a, o); }
};

typedef float wmf_v2f __attribute__((ext_vector_type(2)));

// WMF_XCD: blocks b, b + 8, b + 16 ... run on one XCD (one L2), so give each
// XCD a contiguous run of row-major tiles; the 22x22 regions of horizontally
// adjacent tiles (8 apart) then overlap inside one L2 instead of eight
#ifndef WMF_XCD
#define WMF_XCD 1
#endif

// weight of region sample s for a pixel of guide colour (c01, c2):
// max(2^(nk |dlab|^2) occ, 1e-10), channels 0-1 in packed fp32.  Called from
// the window pass and the chunk walk: both must round identically, so no
// contraction beyond the explicit fma.
__device__ __forceinline__ float wmf_w(const float4 &s, wmf_v2f c01, float c2, float nk) {
#pragma clang fp contract(off)
  const wmf_v2f e = wmf_v2f{s.x, s.y} - c01, q = e * e;
  const float e2 = s.z - c2;
  return fmaxf(__builtin_amdgcn_exp2f(__builtin_fmaf(e2, e2, q.x + q.y) * nk) * s.w, 1e-10f);
}
__device__ __forceinline__ float wmf_w(const float2 &s, wmf_v2f c01, float, float nk) {
#pragma clang fp contract(off)
  const float e = s.x - c01.x;
  return fmaxf(__builtin_amdgcn_exp2f(e * e * nk) * s.y, 1e-10f);
}

// v from lane ^ lj: DPP for lj = 1, 2 (quad_perm), 4 (row_half_mirror then
// quad_perm) and 8 (row_ror:8), a ds_bpermute otherwise (16 and 32 use
// swap_lane64 below) (lj is a constant once the sort loops are unrolled)
__device__ __forceinline__ uint64_t xor_lane64(uint64_t v, int lj) {
  const int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
  int a, b;
  if (lj == 1) {
    a = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xf, 0xf, false);
    b = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xf, 0xf, false);
  } else if (lj == 2) {
    a = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xf, 0xf, false);
    b = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xf, 0xf, false);
  } else if (lj == 8) {
    a = __builtin_amdgcn_mov_dpp(lo, 0x128, 0xf, 0xf, false);
    b = __builtin_amdgcn_mov_dpp(hi, 0x128, 0xf, 0xf, false);
  } else if (lj == 4) {  // row_half_mirror (l ^ 7), then quad_perm [3,2,1,0] (l ^ 3)
    a = __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(lo, 0x141, 0xf, 0xf, false), 0x1B, 0xf, 0xf, false);
    b = __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(hi, 0x141, 0xf, 0xf, false), 0x1B, 0xf, 0xf, false);
  } else {
    return __shfl_xor(v, lj);
  }
  return ((uint64_t)(uint32_t)b << 32) | (uint32_t)a;
}

// (own, partner) of lane ^ lj for lj = 16 / 32 in unspecified order per lane:
// v_permlane16_swap / v_permlane32_swap (gfx950) of each 32-bit half with itself
__device__ __forceinline__ void swap_lane64(uint64_t v, int lj, uint64_t &a, uint64_t &b) {
  const unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
  unsigned alo, blo, ahi, bhi;
  if (lj == 16) {
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    alo = l[0]; blo = l[1]; ahi = h[0]; bhi = h[1];
  } else {
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    alo = l[0]; blo = l[1]; ahi = h[0]; bhi = h[1];
  }
  a = ((uint64_t)ahi << 32) | alo;
  b = ((uint64_t)bhi << 32) | blo;
}

// v_permlane16_swap / v_permlane32_swap of two 64-bit registers: the upper
// row of each 32-lane row pair (lj = 16) / the upper 32 lanes (lj = 32) of x
// trade places with the lower row / half of y, i.e. afterwards lower lanes
// hold (x own, x of lane + lj) and upper lanes (y of lane - lj, y own)
__device__ __forceinline__ void swap_rows64(uint64_t &x, uint64_t &y, int lj) {
  const unsigned xl = (unsigned)x, xh = (unsigned)(x >> 32), yl = (unsigned)y, yh = (unsigned)(y >> 32);
  unsigned a0, a1, b0, b1;
  if (lj == 16) {
    const auto l = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
    a0 = l[0]; b0 = l[1]; a1 = h[0]; b1 = h[1];
  } else {
    const auto l = __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
    a0 = l[0]; b0 = l[1]; a1 = h[0]; b1 = h[1];
  }
  x = ((uint64_t)a1 << 32) | a0;
  y = ((uint64_t)b1 << 32) | b0;
}
#ifndef WMF_SWAP_PAIR
#define WMF_SWAP_PAIR 1
#endif

// Sort keys: the flow value widened to fp64 (exact), the region position
// (ry << 8 | rx) in the 29 mantissa bits the widening leaves zero.  As
// doubles they order by value, ties by position (reversed for negative
// values: any fixed tie order gives the same weighted median), -0 before +0
// like the old integer key; +-inf and NaN map to +-2^1000 / 2^1001 (above
// every finite fp32) so no key is a NaN, padding to 2^1002.  The position is
// the key's low 16 bits either way.
__device__ __forceinline__ uint64_t wmf_key(float v, unsigned pos) {
  // selects, not branches: the region load issues every read before the
  // first key is formed
  const double d = (double)v;
  const double e = v > 0.f ? 0x1p1000 : -0x1p1000;
  const double f = __builtin_isnan(v) ? 0x1p1001 : (__builtin_isinf(v) ? e : d);
  return __builtin_bit_cast(uint64_t, f) | (uint64_t)pos;
}
// padding keys: above every value; position (RW, 0), one row below the
// region -- out of every lane's window (dy = RW - py > 2 hsz), yet its
// record address (RW * RP) is inside the LDS allocation, so the chunk walk
// reads it without a select
#define WMF_PAD_KEY(RW) (__builtin_bit_cast(uint64_t, 0x1p1002) | ((uint64_t)(RW) << 8))
__device__ __forceinline__ double wmf_d(uint64_t k) { return __builtin_bit_cast(double, k); }
// v_min_f64 / v_max_f64 without the canonicalising v_max_f64 x, x that the
// builtins add in IEEE mode (keys are never NaN, and fp64 denormals -- the
// keys of +-0 -- are preserved: float_denorm_mode_16_64 = 3)
__device__ __forceinline__ uint64_t wmf_min(uint64_t a, uint64_t b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(wmf_d(a)), "v"(wmf_d(b)));
  return __builtin_bit_cast(uint64_t, r);
}
__device__ __forceinline__ uint64_t wmf_max(uint64_t a, uint64_t b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(wmf_d(a)), "v"(wmf_d(b)));
  return __builtin_bit_cast(uint64_t, r);
}

// (min, max) of a pair from one asm statement: a select between two outputs
// of one statement cannot be turned into a branch around either
__device__ __forceinline__ void wmf_minmax(uint64_t a, uint64_t b, uint64_t &mn, uint64_t &mx) {
  double r0, r1;
  asm("v_min_f64 %0, %2, %3\n\tv_max_f64 %1, %2, %3" : "=&v"(r0), "=&v"(r1) : "v"(wmf_d(a)), "v"(wmf_d(b)));
  mn = __builtin_bit_cast(uint64_t, r0);
  mx = __builtin_bit_cast(uint64_t, r1);
}
// min(a, -b) in one v_min_f64 (source negate modifier)
__device__ __forceinline__ uint64_t wmf_min_neg(uint64_t a, uint64_t b) {
  double r;
  asm("v_min_f64 %0, %1, -%2" : "=v"(r) : "v"(wmf_d(a)), "v"(wmf_d(b)));
  return __builtin_bit_cast(uint64_t, r);
}

template <int NPER>
struct Bitonic {
  static constexpr int N = NPER * 64;
  // lane bits of the sign in stage (kk, jj): (lane * NPER) & kk, xor lj for a
  // DPP cross-lane stage; and the bit of r (kk < NPER)
  static constexpr int lane_sel(int kk, int jj) {
    return ((kk >= NPER ? kk / NPER : 0) ^ (jj >= NPER && jj / NPER < 16 ? jj / NPER : 0)) & 63;
  }
  static constexpr bool r_bit(int r, int kk) { return kk < NPER && (r & kk) != 0; }

  // one stage (kk, jj) after stage (pkk, pjj) (pkk = 0: none), then the next
  template <int KK, int JJ, int PKK, int PJJ>
  __device__ __forceinline__ static void stage(uint64_t (&ka)[NPER], uint64_t (&kb)[NPER], int lane) {
    constexpr int ls = lane_sel(KK, JJ) ^ (PKK ? lane_sel(PKK, PJJ) : 0);
    const unsigned lflip = ls ? (unsigned)(__builtin_popcount(lane & ls) & 1) << 31 : 0u;
#pragma unroll
    for (int r = 0; r < NPER; ++r) {
      const bool rf = r_bit(r, KK) != (PKK ? r_bit(r, PKK) : false);
      if (ls || rf) {
        const uint64_t m = (uint64_t)(lflip ^ (rf ? 0x80000000u : 0u)) << 32;
        ka[r] ^= m;
        kb[r] ^= m;
      }
    }
    if constexpr (JJ >= NPER) {
      constexpr int lj = JJ / NPER;
      if constexpr (lj == 16 || lj == 32) {
#if WMF_SWAP_PAIR
        // the two lists' key r in one exchange: swap_rows64(a, b) leaves the
        // lower rows / half holding list a's pair (own, partner) and the upper
        // ones list b's pair; each lane forms (min, max) of its pair, and the
        // same exchange of (min, max) hands every lane its own result -- list
        // a: lower min, upper max; list b likewise -- in 3 instructions per
        // key instead of 2 copies + 2 swaps + min + max + 2 selects
#pragma unroll
        for (int r = 0; r < NPER; ++r) {
          uint64_t x = ka[r], y = kb[r], mn, mx;
          swap_rows64(x, y, lj);
          wmf_minmax(x, y, mn, mx);
          swap_rows64(mn, mx, lj);
          ka[r] = mn;
          kb[r] = mx;
        }
#else
        const bool take_min = (lane & lj) == 0;
#pragma unroll
        for (int r = 0; r < NPER; ++r) {
          uint64_t p0, p1, q0, q1, an, ax, bn, bx;
          swap_lane64(ka[r], lj, p0, p1);
          swap_lane64(kb[r], lj, q0, q1);
          wmf_minmax(p0, p1, an, ax);
          wmf_minmax(q0, q1, bn, bx);
          ka[r] = take_min ? an : ax;
          kb[r] = take_min ? bn : bx;
        }
#endif
      } else {
        // every partner first, then the minima: the DPP moves of a key are
        // not right behind the v_xor that wrote it (VALU -> DPP hazard nops)
        uint64_t pa[NPER], pb[NPER];
#pragma unroll
        for (int r = 0; r < NPER; ++r) {
          pa[r] = xor_lane64(ka[r], lj);
          pb[r] = xor_lane64(kb[r], lj);
        }
#pragma unroll
        for (int r = 0; r < NPER; ++r) {
          ka[r] = wmf_min_neg(ka[r], pa[r]);
          kb[r] = wmf_min_neg(kb[r], pb[r]);
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < NPER; ++r) {
        const int rp = r ^ JJ;
        if (rp > r) {
          const uint64_t a0 = ka[r], a1 = ka[rp], b0 = kb[r], b1 = kb[rp];
          ka[r] = wmf_min(a0, a1);
          ka[rp] = wmf_max(a0, a1);
          kb[r] = wmf_min(b0, b1);
          kb[rp] = wmf_max(b0, b1);
        }
      }
    }
    if constexpr (JJ > 1) {
      stage<KK, JJ / 2, KK, JJ>(ka, kb, lane);
    } else if constexpr (KK < N) {
      stage<2 * KK, KK, KK, JJ>(ka, kb, lane);
    } else {
      // back to plain keys (the last merge's blocks are all ascending and
      // its last stage is in-lane: nothing left to flip unless NPER == 1)
      constexpr int le = lane_sel(KK, JJ);
      if constexpr (le != 0) {
        const uint64_t m = (uint64_t)((unsigned)(__builtin_popcount(lane & le) & 1) << 31) << 32;
#pragma unroll
        for (int r = 0; r < NPER; ++r) {
          ka[r] ^= m;
          kb[r] ^= m;
        }
      }
    }
  }
};

// Bitonic sort of the 64*NPER keys of two lists at once (element e = lane *
// NPER + r).  Merge kk sorts blocks of kk elements ascending where e & kk is
// 0 and descending elsewhere; the keys of descending blocks carry a flipped
// sign bit during that merge (min of negated keys = max), so every
// compare-exchange is ascending.  A pair inside a lane is one v_min_f64 + one
// v_max_f64.  A pair across lanes at lane distance lj < 16 (DPP partner):
// during that stage the upper lane of each pair (lane & lj) holds its keys
// negated as well, so both lanes compute min(own, -partner) -- the lower lane
// gets min(x_L, x_U), the upper -max(x_L, x_U) -- one v_min_f64 with a
// negated source and no per-lane select (was v_cmp + an SALU xor of the
// compare mask with the lane's direction + two v_cndmask, the compare mask
// one SGPR pair every key waited on).  The sign changes between stages are
// one v_xor of the high dword per key with a lane-only mask (Bitonic::stage:
// every stage a template instance, so every mask and partner distance is a
// compile-time constant).  At lj = 16 / 32 (v_permlane{16,32}_swap: own and
// partner in a lane-dependent order) both lanes form min and max and keep
// one by a lane-constant mask.
template <int NPER>
__device__ __forceinline__ void bitonic_regs2(uint64_t (&ka)[NPER], uint64_t (&kb)[NPER], int lane) {
  Bitonic<NPER>::template stage<2, 1, 0, 0>(ka, kb, lane);
}

// HS > 0: area_hsz fixed at compile time (window loop fully unrolled,
// immediate LDS offsets); HS == 0: runtime hsz.  RP = LDS row pitch of the
// region records (RP % 16 == 8: the 8 rows of a tile fall on disjoint banks).
// LDS (not VGPRs) bounds the occupancy at 2 waves per SIMD: let the
// scheduler use the registers to keep LDS reads in flight
template <int GC, int NPER, int HS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_wmf(const float2 *__restrict__ uv, const float *__restrict__ guide,
                                             const float *__restrict__ occ, float2 *out, int H, int W,
                                             int P, size_t ps, int hsz_rt, float nk, int RW_rt, int RP_rt,
                                             const float2 *base) {
  using T = typename WmfRec<GC>::T;
  constexpr int N = NPER * 64, NC = wmf_nc(N), CH = N / NC;
  const int hsz = HS > 0 ? HS : hsz_rt;
  // region width and record pitch: compile-time with HS (no runtime divides)
  constexpr int RWc = WMF_T + 2 * HS, RPc = RWc + ((8 - RWc) % 16 + 16) % 16;
  const int RW = HS > 0 ? RWc : RW_rt, RP = HS > 0 ? RPc : RP_rt;
  // whole-sample reflect with one fold reaches every region sample when the
  // plane has >= WMF_T + hsz rows / columns (all pyramid levels of the
  // registry); otherwise the general modulo form
  const bool fold1 = H >= WMF_T + hsz && W >= WMF_T + hsz;
  auto mir = [&](int i, int n) { return fold1 ? (i < 0 ? -i : (i >= n ? 2 * (n - 1) - i : i)) : ext_mirror(i, n); };
  const int nreg = RW * RW;
  // LDS: chunk sums [2][WMF_NC][64] f64 (u chunks, then v chunks; a chunk's
  // 64 lane slots are contiguous, so a scatter-add never conflicts) | records
  // [RW][RP] | sorted positions (ry << 8 | rx) of the u and v lists [2][N] u16 |
  // chunk ids [RW][RP][2] u8 (u list, v list of a sample side by side: the
  // window pass reads both with one u16 load)
  extern __shared__ double lds_f64[];
  wmf_sum_t *csum = reinterpret_cast<wmf_sum_t *>(lds_f64);
  T *smp = reinterpret_cast<T *>(csum + 2 * NC * 64);
  uint16_t *ku = reinterpret_cast<uint16_t *>(smp + RW * RP), *kv = ku + N;
  uint8_t *cid = reinterpret_cast<uint8_t *>(kv + N);
  int tbx = blockIdx.x, tby = blockIdx.y;
  if (WMF_XCD) {
    const int nt = gridDim.x * gridDim.y, lin = blockIdx.x + blockIdx.y * gridDim.x;
    const int xcd = lin & 7, tile = xcd * (nt >> 3) + min(xcd, nt & 7) + (lin >> 3);
    tby = tile / gridDim.x;
    tbx = tile - tby * gridDim.x;
  }
  const int ty0 = tby * WMF_T, tx0 = tbx * WMF_T;
  const int lane = threadIdx.x;
  WMF_STAMP(0);
  // region load: every lane's NPER samples' offsets first (padding lanes,
  // s >= nreg, re-read the last sample and rewrite its record with the same
  // bytes), then all uv / guide / occ reads, then keys and records -- no
  // branch between the reads, so they are all in flight at once (was one
  // round trip per sample and read kind: 15.5 K of 102 K cycles per wave)
  uint64_t a[NPER], b[NPER];
  unsigned goff[NPER], rpos[NPER];
  auto region_offsets = [&](auto mirf) {
#pragma unroll
    for (int r = 0; r < NPER; ++r) {
      const int s = min(lane * NPER + r, nreg - 1);
      const int ry = s / RW, rx = s - ry * RW;
      goff[r] = (unsigned)(mirf(ty0 - hsz + ry, H) * P + mirf(tx0 - hsz + rx, W));
      rpos[r] = ((unsigned)ry << 8) | (unsigned)rx;
    }
  };
  if (fold1)
    region_offsets([](int i, int n) { return i < 0 ? -i : (i >= n ? 2 * (n - 1) - i : i); });
  else
    region_offsets([](int i, int n) { return ext_mirror(i, n); });
  float2 rv[NPER];
  float rg[NPER][3], ro[NPER];
#pragma unroll
  for (int r = 0; r < NPER; ++r) rv[r] = uv[goff[r]];
#pragma unroll
  for (int r = 0; r < NPER; ++r) {
#pragma unroll
    for (int c = 0; c < 3; ++c) rg[r][c] = c < GC ? guide[c * ps + goff[r]] : 0.f;
    ro[r] = occ[goff[r]];
  }
#pragma unroll
  for (int r = 0; r < NPER; ++r) {
    // padding keys by a mask, not a select: a per-lane select lets the
    // compiler sink the last sample's read into a branch behind the others
    const uint64_t pm = 0ull - (uint64_t)(lane * NPER + r >= nreg);
    const uint64_t ka = wmf_key(rv[r].x, rpos[r]), kb = wmf_key(rv[r].y, rpos[r]);
    a[r] = ka ^ ((ka ^ WMF_PAD_KEY(RW)) & pm);
    b[r] = kb ^ ((kb ^ WMF_PAD_KEY(RW)) & pm);
    smp[(rpos[r] >> 8) * RP + (rpos[r] & 0xffu)] = WmfRec<GC>::make(rg[r][0], rg[r][1], rg[r][2], ro[r]);
  }
  wmf_sum_t *cs = csum + lane;
#pragma unroll
  for (int c = 0; c < 2 * NC; ++c) cs[c * 64] = 0.0;
  WMF_STAMP(1);
  bitonic_regs2<NPER>(a, b, lane);
#pragma unroll
  for (int r = 0; r < NPER; ++r) {
    const int e = lane * NPER + r;
    const unsigned pa = (uint16_t)a[r], pb = (uint16_t)b[r];
    ku[e] = (uint16_t)pa;  // padding keys -> (RW, 0): out of every window
    kv[e] = (uint16_t)pb;
    const int qa = (pa >> 8) * RP + (pa & 0xffu), qb_ = (pb >> 8) * RP + (pb & 0xffu);
    const unsigned padpos = (unsigned)RW << 8;
    if (pa != padpos) cid[WMF_CID_PAIR ? 2 * qa : qa] = (uint8_t)(e / CH);
    if (pb != padpos) cid[WMF_CID_PAIR ? 2 * qb_ + 1 : RW * RP + qb_] = (uint8_t)(e / CH);
  }
  __syncthreads();
  WMF_STAMP(2);
  const int py = lane >> 3, px = lane & 7;
  const int gi = ty0 + py, gj = tx0 + px;
  const int qb = py * RP + px;
  float cg[3] = {0.f, 0.f, 0.f};
  {
    const T c0 = smp[qb + hsz * RP + hsz];
    const float *cf = reinterpret_cast<const float *>(&c0);
#pragma unroll
    for (int c = 0; c < GC; ++c) cg[c] = cf[c];
  }
  const wmf_v2f c01 = {cg[0], cg[1]};
  // window pass: the per-chunk weight of both lists.  One window row per
  // step: its records and chunk offsets are read first, so the LDS latency
  // is paid once per row.
  char *csb = reinterpret_cast<char *>(cs);
  auto visit_row = [&](int q0, int n) {
    constexpr int MX = HS > 0 ? 2 * HS + 1 : 5;
    T rec[MX];
    unsigned cu[MX], cv[MX];
#pragma unroll
    for (int dx = 0; dx < MX; ++dx)
      if (dx < n) {
        rec[dx] = smp[q0 + dx];
        if (WMF_CID_PAIR) {
          const unsigned pr = reinterpret_cast<const uint16_t *>(cid)[q0 + dx];
          cu[dx] = pr & 0xffu;
          cv[dx] = pr >> 8;
        } else {
          cu[dx] = cid[q0 + dx];
          cv[dx] = cid[RW * RP + q0 + dx];
        }
      }
#pragma unroll
    for (int dx = 0; dx < MX; ++dx)
      if (dx < n) {
        const wmf_sum_t w = (wmf_sum_t)wmf_w(rec[dx], c01, cg[2], nk);
        atomicAdd(reinterpret_cast<wmf_sum_t *>(csb + (cu[dx] << WMF_SUM_SHIFT)), w);
        atomicAdd(reinterpret_cast<wmf_sum_t *>(csb + (cv[dx] << WMF_SUM_SHIFT)) + NC * 64, w);
      }
  };
  if (HS > 0) {
#pragma unroll
    for (int dy = 0; dy <= 2 * HS; ++dy) visit_row(qb + dy * RP, 2 * HS + 1);
  } else {
    for (int dy = 0; dy <= 2 * hsz; ++dy)
      for (int dx = 0; dx <= 2 * hsz; dx += 5) visit_row(qb + dy * RP + dx, min(5, 2 * hsz + 1 - dx));
  }
  WMF_STAMP(3);
  double su[NC], sv[NC], tot = 0.0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    su[c] = cs[c * 64];
    sv[c] = cs[(NC + c) * 64];
    tot += su[c];
  }
  const double half = 0.5 * tot;
  // crossing chunk of each list: first chunk whose running sum reaches half
  double pu = 0.0, pv = 0.0, bu = 0.0, bv = 0.0;
  int chu = -1, chv = -1, lastu = 0, lastv = 0;
  double lbu = 0.0, lbv = 0.0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (chu < 0 && su[c] > 0.0) { lastu = c; lbu = pu; }
    if (chv < 0 && sv[c] > 0.0) { lastv = c; lbv = pv; }
    if (chu < 0 && pu + su[c] >= half) { chu = c; bu = pu; }
    if (chv < 0 && pv + sv[c] >= half) { chv = c; bv = pv; }
    pu += su[c];
    pv += sv[c];
  }
  // rounding of the v chunk sums vs the total: fall back to the last chunk
  // with window weight (the walk then ends on its last window sample)
  if (chu < 0) { chu = lastu; bu = lbu; }
  if (chv < 0) { chv = lastv; bv = lbv; }
  WMF_STAMP(4);
  const unsigned span = 2u * hsz;
  // walk results as record indices relative to the lane's window origin qb
#if WMF_WALK_LAST
  // The median is the first in-window sample whose cumulative sum reaches
  // half; every in-window weight is >= 1e-10 (far above an ulp of a sum
  // <= 225), so the sums strictly increase and that sample is also the LAST
  // in-window sample whose sum BEFORE it is still below half (the walk starts
  // below half: the crossing chunk's prefix, or the fallback's).  With no
  // crossing in the chunk that is its last in-window sample -- the fallback
  // below -- so one compare and one select per sample and list, no "found"
  // state (the same sample bitwise; the first-reach form: WMF_WALK_LAST 0)
  unsigned resu = 0, resv = 0;
#else
  unsigned resu = 0xffffu, resv = 0xffffu, lstu = 0, lstv = 0;  // 0xffff: none yet
#endif
  // the crossing chunks' sorted positions (ry << 8 | rx), 8 per 16-B read;
  // window offsets straight from the position bytes (dy = ry - py and
  // dx = rx - px as unsigned: out of the window unless both <= span; padding
  // keys have ry = RW)
  const uint4 *wu = reinterpret_cast<const uint4 *>(ku + chu * CH), *wv = reinterpret_cast<const uint4 *>(kv + chv * CH);
  for (int g = 0; g < CH / 8; ++g) {
    const uint4 A = wu[g], B = wv[g];
    const unsigned wa4[4] = {A.x, A.y, A.z, A.w}, wb4[4] = {B.x, B.y, B.z, B.w};
    unsigned qa[8], qv[8];
    bool ina[8], inb[8];
    T ra[8], rb[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int sh = 16 * (i & 1);
      const unsigned wa = wa4[i >> 1], wb = wb4[i >> 1];
      const unsigned dya = ((wa >> (sh + 8)) & 0xffu) - (unsigned)py, dxa = ((wa >> sh) & 0xffu) - (unsigned)px;
      const unsigned dyb = ((wb >> (sh + 8)) & 0xffu) - (unsigned)py, dxb = ((wb >> sh) & 0xffu) - (unsigned)px;
      ina[i] = max(dya, dxa) <= span;
      inb[i] = max(dyb, dxb) <= span;
      // qb + qa = ry * RP + rx: inside the region for every real sample, the
      // word after it for a padding key (no select needed for the read)
      qa[i] = dya * (unsigned)RP + dxa;
      qv[i] = dyb * (unsigned)RP + dxb;
      ra[i] = smp[qb + qa[i]];
      rb[i] = smp[qb + qv[i]];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float xa = wmf_w(ra[i], c01, cg[2], nk), xb = wmf_w(rb[i], c01, cg[2], nk);
#if WMF_WALK_LAST
      resu = (ina[i] && bu < half) ? qa[i] : resu;
      resv = (inb[i] && bv < half) ? qv[i] : resv;
#endif
      // select before the widening: one v_cndmask instead of two (the empty
      // asm keeps the compiler from hoisting the conversion above the select)
      float sa = ina[i] ? xa : 0.f, sb = inb[i] ? xb : 0.f;
      asm("" : "+v"(sa), "+v"(sb));
      bu += (double)sa;
      bv += (double)sb;
#if !WMF_WALK_LAST
      resu = (resu == 0xffffu && ina[i] && bu >= half) ? qa[i] : resu;
      resv = (resv == 0xffffu && inb[i] && bv >= half) ? qv[i] : resv;
      lstu = ina[i] ? qa[i] : lstu;
      lstv = inb[i] ? qv[i] : lstv;
#endif
    }
    // (measured r5v: a wave-level exit once every lane has both medians,
    // `if (!__any(resu == 0xffff || resv == 0xffff)) break;`, is 1.5 % slower
    // per launch, 0.812 vs 0.801 ms, same flow: the walk is short and the
    // vote costs more than the samples it saves)
  }
#if !WMF_WALK_LAST
  if (resu == 0xffffu) resu = lstu;
  if (resv == 0xffffu) resv = lstv;
#endif
  WMF_STAMP(5);
  if (gi < H && gj < W) {
    // the selected samples' values, re-read at their (mirrored) positions
    const int dya = (int)(resu / (unsigned)RP), dyb = (int)(resv / (unsigned)RP);
    const int ya = mir(gi - hsz + dya, H), xa = mir(gj - hsz + (int)resu - dya * RP, W);
    const int yb = mir(gi - hsz + dyb, H), xb = mir(gj - hsz + (int)resv - dyb * RP, W);
    float2 med = make_float2(uv[(size_t)ya * P + xa].x, uv[(size_t)yb * P + xb].y);
    if (base) {  // out = base + (med - base): classic_nl.py:271-275 fused (out may alias base)
      const float2 b0 = base[(size_t)gi * P + gj];
      med = make_float2(b0.x + (med.x - b0.x), b0.y + (med.y - b0.y));
    }
    out[(size_t)gi * P + gj] = med;
  }
}

#define OF_WMF(GC, NP, HS)                                                                                       \
  template __global__ void k_wmf<GC, NP, HS>(const float2 *, const float *, const float *, float2 *, int, int, int, \
                                              size_t, int, float, int, int, const float2 *);
OF_WMF(1, 1, 0) OF_WMF(1, 2, 0) OF_WMF(1, 4, 0) OF_WMF(1, 8, 0) OF_WMF(1, 16, 0) OF_WMF(1, 8, 7)
OF_WMF(3, 1, 0) OF_WMF(3, 2, 0) OF_WMF(3, 4, 0) OF_WMF(3, 8, 0) OF_WMF(3, 16, 0) OF_WMF(3, 8, 7)
#undef OF_WMF
