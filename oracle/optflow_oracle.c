/*
 * optflow_oracle.c — TEST INFRASTRUCTURE, NOT PRODUCT CODE.
 *
 * A float64 CPU restatement of jordanshivers/optical-flow-python's hot path
 * (SURVEY.md §8a rows a1-a18), used only by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg as the parity checker.  The product path
 * (optical_flow -> liboptflow.so, HIP) never links or calls this file.
 *
 * Parity of this restatement is pinned by the golden vectors in tests/golden/
 * (generated from the reference itself by tests/golden/gen_golden.py) and by
 * scipy.ndimage for the third-party primitives the reference calls.
 *
 * Every function cites the reference file:line it restates.  Layout: planar
 * row-major float64 (plane c of an HxW image at c*H*W), flow = u plane, v
 * plane.  OpenMP parallelises pixel loops only; results do not depend on the
 * thread count (no reductions are split across threads except the solver dot
 * products, which use a fixed static partition).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "optflow.h"

#define IDX(i, j, W) ((long)(i) * (W) + (j))

/* ------------------------------------------------------------------ */
/* boundary extensions                                                 */
/* ------------------------------------------------------------------ */
/* scipy.ndimage mode='reflect' (half-sample symmetric, d c b a | a b c d) */
static inline int ext_reflect(int i, int n) {
  if (n == 1) return 0;
  int p = 2 * n;
  i %= p;
  if (i < 0) i += p;
  return i < n ? i : p - 1 - i;
}
/* np.pad mode='reflect' / scipy 'mirror' (whole-sample, d c b | a b c d) */
static inline int ext_mirror(int i, int n) {
  if (n == 1) return 0;
  int p = 2 * (n - 1);
  i %= p;
  if (i < 0) i += p;
  return i < n ? i : p - i;
}
static inline int clampi(int i, int lo, int hi) { return i < lo ? lo : (i > hi ? hi : i); }

/* ------------------------------------------------------------------ */
/* robust penalties: optical_flow/robust/penalties.py:18-345           */
/* ------------------------------------------------------------------ */
double ofr_penalty(int kind, double p0, double p1, double x, int d) {
  switch (kind) {
    case OF_PEN_QUADRATIC: { /* penalties.py:18-41 */
      double s2 = p0 * p0;
      return d == 0 ? x * x / s2 : d == 1 ? 2.0 * x / s2 : 2.0 / s2;
    }
    case OF_PEN_LORENTZIAN: { /* :44-67 */
      double s2 = p0 * p0;
      return d == 0 ? log(1.0 + x * x / (2.0 * s2)) : d == 1 ? 2.0 * x / (2.0 * s2 + x * x) : 2.0 / (2.0 * s2 + x * x);
    }
    case OF_PEN_CHARBONNIER: { /* :70-102 */
      double s2 = p0 * p0, t = x / s2, sr = sqrt(1.0 + t * t);
      return d == 0 ? s2 * sr : d == 1 ? x / (s2 * sr) : 1.0 / (s2 * sr);
    }
    case OF_PEN_GEN_CHARBONNIER: { /* :105-131 */
      double base = p0 * p0 + x * x;
      return d == 0 ? pow(base, p1) : d == 1 ? 2.0 * p1 * x * pow(base, p1 - 1.0) : 2.0 * p1 * pow(base, p1 - 1.0);
    }
    case OF_PEN_GEMAN_MCCLURE: { /* :134-158 */
      double s2 = p0 * p0, den = s2 + x * x;
      return d == 0 ? x * x / den : d == 1 ? 2.0 * s2 * x / (den * den) : 2.0 * s2 / (den * den);
    }
    case OF_PEN_HUBER: { /* :161-198 */
      double s2 = p0 * p0, ax = fabs(x);
      int in = ax <= s2;
      if (d == 0) return in ? x * x : 2.0 * s2 * ax - s2 * s2;
      if (d == 1) return in ? 2.0 * x : 2.0 * s2 * (x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0));
      return in ? 2.0 : 2.0 * s2 / fmax(ax, 1e-30);
    }
    case OF_PEN_TUKEY: { /* :201-240 */
      double s2 = p0 * p0, om = 1.0 - x * x / s2;
      int in = fabs(x) <= p0;
      if (d == 0) return in ? (1.0 / 3.0) * (1.0 - om * om * om) : 1.0 / 3.0;
      if (d == 1) return in ? 2.0 * x * om * om / s2 : 0.0;
      return in ? 2.0 * om * om / s2 : 0.0;
    }
    case OF_PEN_GAUSSIAN: { /* :243-268 */
      double s2 = p0 * p0;
      if (d == 0) return 0.5 * log(2.0 * M_PI) + log(p0) + 0.5 * (x / p0) * (x / p0);
      return d == 1 ? x / s2 : 1.0 / s2;
    }
    case OF_PEN_TDIST:
    case OF_PEN_TDIST_UNNORM: { /* :271-345 */
      double r = p0, s = p1, s2r = s * s * r;
      if (d == 0) {
        double y = (r + 1.0) / 2.0 * log(1.0 + x * x / s2r);
        if (kind == OF_PEN_TDIST) y += lgamma(r / 2.0) - lgamma((r + 1.0) / 2.0) + 0.5 * log(r * M_PI) + log(s);
        return y;
      }
      return d == 1 ? (r + 1.0) * x / (s2r + x * x) : (r + 1.0) / (s2r + x * x);
    }
    case OF_PEN_CONST:
      return d == 2 ? p0 : (d == 1 ? p0 * x : 0.5 * p0 * x * x);
  }
  return NAN;
}

void ofr_penalty_array(int kind, double p0, double p1, int d, const double *x, double *y, long n) {
  for (long i = 0; i < n; ++i) y[i] = ofr_penalty(kind, p0, p1, x[i], d);
}
static inline double pen_w(const of_penalty *p, double x) { return ofr_penalty(p->kind, p->p0, p->p1, x, 2); }

/* ------------------------------------------------------------------ */
/* preprocessing: interface.py:74-141, image_processing.py:6-49        */
/* ------------------------------------------------------------------ */
/* _rgb2gray (interface.py:74-88); rgb interleaved HxWx3 */
void ofr_rgb2gray(const double *rgb, int H, int W, double *gray) {
  long n = (long)H * W;
  for (long k = 0; k < n; ++k) {
    double c[3];
    for (int t = 0; t < 3; ++t) {
      double q = floor(rgb[3 * k + t] + 0.5);
      q = q < 0 ? 0 : (q > 255 ? 255 : q);
      c[t] = (double)(unsigned char)q;
    }
    gray[k] = floor(0.2989 * c[0] + 0.5870 * c[1] + 0.1140 * c[2] + 0.5);
  }
}

/* _rgb2lab (interface.py:91-141); output planar L,a,b */
void ofr_rgb2lab(const double *rgb, int H, int W, double *lab) {
  long n = (long)H * W;
  double mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (long k = 0; k < n; ++k)
    for (int t = 0; t < 3; ++t) mx[t] = fmax(mx[t], rgb[3 * k + t]);
  int norm = mx[0] > 1.0 || mx[1] > 1.0 || mx[2] > 1.0;
  const double T = 0.008856;
  for (long k = 0; k < n; ++k) {
    double R = rgb[3 * k], G = rgb[3 * k + 1], B = rgb[3 * k + 2];
    if (norm) { R /= 255.0; G /= 255.0; B /= 255.0; }
    double X = (0.412453 * R + 0.357580 * G + 0.180423 * B) / 0.950456;
    double Y = 0.212671 * R + 0.715160 * G + 0.072169 * B;
    double Z = (0.019334 * R + 0.119193 * G + 0.950227 * B) / 1.088754;
    double Y3 = cbrt(Y);
    double fX = X > T ? cbrt(X) : 7.787 * X + 16.0 / 116.0;
    double fY = Y > T ? Y3 : 7.787 * Y + 16.0 / 116.0;
    double fZ = Z > T ? cbrt(Z) : 7.787 * Z + 16.0 / 116.0;
    lab[k] = Y > T ? 116.0 * Y3 - 16.0 : 903.3 * Y;
    lab[n + k] = 500.0 * (fX - fY);
    lab[2 * n + k] = 200.0 * (fY - fZ);
  }
}

/* scale_image (image_processing.py:6-26), min/max over all n values */
void ofr_scale_image(double *im, long n, double vlow, double vhigh) {
  double lo = INFINITY, hi = -INFINITY;
  for (long k = 0; k < n; ++k) { lo = fmin(lo, im[k]); hi = fmax(hi, im[k]); }
  if (hi == lo) { for (long k = 0; k < n; ++k) im[k] = (vlow + vhigh) / 2.0; return; }
  for (long k = 0; k < n; ++k) im[k] = (im[k] - lo) / (hi - lo) * (vhigh - vlow) + vlow;
}

/* fspecial_gaussian (image_processing.py:29-49) */
void ofr_gaussian(int size, double sigma, double *k) {
  double m = (size - 1) / 2.0, mx = 0, s = 0;
  for (int a = 0; a < size; ++a)
    for (int b = 0; b < size; ++b) {
      double y = a - m, x = b - m;
      k[a * size + b] = exp(-(x * x + y * y) / (2 * sigma * sigma));
      mx = fmax(mx, k[a * size + b]);
    }
  for (int t = 0; t < size * size; ++t) { if (k[t] < DBL_EPSILON * mx) k[t] = 0; s += k[t]; }
  if (s != 0) for (int t = 0; t < size * size; ++t) k[t] /= s;
}

/* _rof_structure_2d (image_processing.py:86-136) */
static void rof_structure_2d(const double *im, int H, int W, double theta, int iters, double *out) {
  long n = (long)H * W;
  double *p0 = calloc(n, sizeof(double)), *p1 = calloc(n, sizeof(double));
  double *u = malloc(n * sizeof(double));
  const double delta = 1.0 / (4.0 * theta);
  for (int it = 0; it <= iters; ++it) {
#pragma omp parallel for schedule(static) if ((long)H * W > 40000)
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < W; ++j) {
        long k = IDX(i, j, W);
        double d = j > 0 ? p0[k] - p0[k - 1] : p0[k];
        d += i > 0 ? p1[k] - p1[k - W] : p1[k];
        u[k] = im[k] + theta * d;
      }
    if (it == iters) break; /* final divergence -> structure (:297-304) */
#pragma omp parallel for schedule(static) if ((long)H * W > 40000)
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < W; ++j) {
        long k = IDX(i, j, W);
        double gx = j < W - 1 ? u[k + 1] - u[k] : 0.0;
        double gy = i < H - 1 ? u[k + W] - u[k] : 0.0;
        double a = p0[k] + delta * gx, b = p1[k] + delta * gy;
        double nrm = sqrt(a * a + b * b);
        nrm = nrm > 1.0 ? nrm : 1.0;
        p0[k] = a / nrm;
        p1[k] = b / nrm;
      }
  }
  memcpy(out, u, n * sizeof(double));
  free(p0); free(p1); free(u);
}

/* structure_texture_decomposition_rof (image_processing.py:52-83); planar C */
void ofr_rof_texture(const double *im, int H, int W, int C, double theta, int iters, double alp, double *out) {
  long n = (long)H * W;
  double *nrm = malloc(n * C * sizeof(double)), *st = malloc(n * sizeof(double));
  memcpy(nrm, im, n * C * sizeof(double));
  ofr_scale_image(nrm, n * C, -1.0, 1.0);
  for (int c = 0; c < C; ++c) {
    rof_structure_2d(nrm + c * n, H, W, theta, iters, st);
    for (long k = 0; k < n; ++k) out[c * n + k] = nrm[c * n + k] - alp * st[k];
  }
  ofr_scale_image(out, n * C, 0.0, 255.0);
  free(nrm); free(st);
}

/* ------------------------------------------------------------------ */
/* filtering / resampling: scipy.ndimage.correlate + map_coordinates    */
/* ------------------------------------------------------------------ */
/* correlate(in, k, mode='reflect'), odd kh x kw kernel centred at (kh/2, kw/2) */
void ofr_correlate(const double *in, int H, int W, const double *k, int kh, int kw, double *out) {
  int ch = kh / 2, cw = kw / 2;
#pragma omp parallel for schedule(static) if ((long)H * W > 40000)
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) {
      double s = 0;
      for (int a = 0; a < kh; ++a) {
        int ii = ext_reflect(i + a - ch, H);
        for (int b = 0; b < kw; ++b) {
          double w = k[a * kw + b];
          if (w == 0.0) continue;
          s += w * in[IDX(ii, ext_reflect(j + b - cw, W), W)];
        }
      }
      out[IDX(i, j, W)] = s;
    }
}

/* bilinear sample with coordinates already clipped to [0,n-1]
 * (map_coordinates order=1 mode='nearest', pyramid.py:35-40, warping.py:41-44) */
static inline double bilin_clamped(const double *a, int H, int W, double r, double c) {
  int i0 = (int)floor(r), j0 = (int)floor(c);
  double fr = r - i0, fc = c - j0;
  int i1 = clampi(i0 + 1, 0, H - 1), j1 = clampi(j0 + 1, 0, W - 1);
  i0 = clampi(i0, 0, H - 1); j0 = clampi(j0, 0, W - 1);
  return (1 - fr) * ((1 - fc) * a[IDX(i0, j0, W)] + fc * a[IDX(i0, j1, W)]) +
         fr * ((1 - fc) * a[IDX(i1, j0, W)] + fc * a[IDX(i1, j1, W)]);
}

/* _matlab_imresize_bilinear to an explicit size (pyramid.py:11-41) */
void ofr_imresize(const double *in, int H, int W, int nH, int nW, double *out) {
  double sH = (double)nH / H, sW = (double)nW / W;
#pragma omp parallel for schedule(static) if ((long)H * W > 40000)
  for (int o = 0; o < nH; ++o) {
    double r = (o + 0.5) / sH - 0.5;
    r = r < 0 ? 0 : (r > H - 1 ? H - 1 : r);
    for (int q = 0; q < nW; ++q) {
      double c = (q + 0.5) / sW - 0.5;
      c = c < 0 ? 0 : (c > W - 1 ? W - 1 : c);
      out[IDX(o, q, nW)] = bilin_clamped(in, H, W, r, c);
    }
  }
}

static inline int matlab_round(double x) { return (int)floor(x + 0.5); }
void ofr_resize_dims(int H, int W, double ratio, int *nH, int *nW) {
  int a = matlab_round(H * ratio), b = matlab_round(W * ratio);
  *nH = a < 1 ? 1 : a;
  *nW = b < 1 ? 1 : b;
}

/* one compute_image_pyramid step (pyramid.py:58-67), planar C channels */
void ofr_pyramid_level(const double *in, int H, int W, int C, const double *k, int ks, double ratio,
                       double *out, int *oH, int *oW) {
  int nH, nW;
  ofr_resize_dims(H, W, ratio, &nH, &nW);
  double *tmp = malloc((long)H * W * sizeof(double));
  for (int c = 0; c < C; ++c) {
    ofr_correlate(in + (long)c * H * W, H, W, k, ks, ks, tmp);
    ofr_imresize(tmp, H, W, nH, nW, out + (long)c * nH * nW);
  }
  free(tmp);
  *oH = nH; *oW = nW;
}

/* resample_flow (warping.py:6-45): both components scaled by the HEIGHT ratio */
void ofr_resample_flow(const double *uv, int H, int W, int nH, int nW, double *out) {
  if (H == nH && W == nW) { memcpy(out, uv, 2L * H * W * sizeof(double)); return; }
  double ratio = (double)nH / H;
  for (int c = 0; c < 2; ++c) {
    ofr_imresize(uv + (long)c * H * W, H, W, nH, nW, out + (long)c * nH * nW);
    for (long k = 0; k < (long)nH * nW; ++k) out[(long)c * nH * nW + k] *= ratio;
  }
}

/* ------------------------------------------------------------------ */
/* warping + derivatives: derivatives.py:27-296                         */
/* ------------------------------------------------------------------ */
/* cubic Hermite basis: the tensor-product form of the 16x16 bicubic
 * coefficient matrix (derivatives.py:7-24, 103-140) */
static inline void hermite_basis(double t, double h[4], double dh[4]) {
  double t2 = t * t, t3 = t2 * t;
  h[0] = 2 * t3 - 3 * t2 + 1; /* value at 0 */
  h[1] = -2 * t3 + 3 * t2;    /* value at 1 */
  h[2] = t3 - 2 * t2 + t;     /* slope at 0 */
  h[3] = t3 - t2;             /* slope at 1 */
  dh[0] = 6 * t2 - 6 * t;
  dh[1] = -6 * t2 + 6 * t;
  dh[2] = 3 * t2 - 4 * t + 1;
  dh[3] = 3 * t2 - 2 * t;
}

/* interp2_bicubic (derivatives.py:27-145) given precomputed DX, DY, DXY grids;
 * XI, YI 1-based query coordinates */
static void interp2_bicubic_pre(const double *Z, const double *DX, const double *DY, const double *DXY,
                                int H, int W, double XI, double YI, double *zi, double *zx, double *zy, int *oob) {
  int fx = (int)floor(XI), fy = (int)floor(YI);
  int cx = fx + 1, cy = fy + 1;
  *oob = (fx < 1) || (cx > W) || (fy < 1) || (cy > H);
  int fx0 = clampi(fx, 1, W) - 1, cx0 = clampi(cx, 1, W) - 1;
  int fy0 = clampi(fy, 1, H) - 1, cy0 = clampi(cy, 1, H) - 1;
  double ax = *oob ? 0.0 : XI - floor(XI), ay = *oob ? 0.0 : YI - floor(YI);
  double hx[4], dhx[4], hy[4], dhy[4];
  hermite_basis(ax, hx, dhx);
  hermite_basis(ay, hy, dhy);
  long c00 = IDX(fy0, fx0, W), c10 = IDX(fy0, cx0, W), c01 = IDX(cy0, fx0, W), c11 = IDX(cy0, cx0, W);
  /* f(ax, ay) = sum over corners of value/slope basis products */
  double v = 0, vx = 0, vy = 0;
  long cs[4] = {c00, c10, c01, c11};
  for (int q = 0; q < 4; ++q) {
    int xi = q & 1, yi = q >> 1;
    double gx = hx[xi], gy = hy[yi], sx = hx[2 + xi], sy = hy[2 + yi];
    double dgx = dhx[xi], dgy = dhy[yi], dsx = dhx[2 + xi], dsy = dhy[2 + yi];
    double z = Z[cs[q]], dx = DX[cs[q]], dy = DY[cs[q]], dxy = DXY[cs[q]];
    v += gx * gy * z + sx * gy * dx + gx * sy * dy + sx * sy * dxy;
    vx += dgx * gy * z + dsx * gy * dx + dgx * sy * dy + dsx * sy * dxy;
    vy += gx * dgy * z + sx * dgy * dx + gx * dsy * dy + sx * dsy * dxy;
  }
  *zi = *oob ? NAN : v;
  *zx = vx;
  *zy = vy;
}

void ofr_deriv_grids(const double *Z, int H, int W, const double *filt, double *DX, double *DY, double *DXY) {
  double kxy[25];
  for (int a = 0; a < 5; ++a)
    for (int b = 0; b < 5; ++b) kxy[a * 5 + b] = filt[a] * filt[b];
  if (DX) ofr_correlate(Z, H, W, filt, 1, 5, DX);
  if (DY) ofr_correlate(Z, H, W, filt, 5, 1, DY);
  if (DXY) ofr_correlate(Z, H, W, kxy, 5, 5, DXY);
}

/* public interp2_bicubic for the fixture test */
void ofr_interp2_bicubic(const double *Z, int H, int W, const double *XI, const double *YI, long n,
                         const double *filt, double *ZI, double *ZXI, double *ZYI) {
  long N = (long)H * W;
  double *DX = malloc(N * sizeof(double)), *DY = malloc(N * sizeof(double)), *DXY = malloc(N * sizeof(double));
  ofr_deriv_grids(Z, H, W, filt, DX, DY, DXY);
  for (long k = 0; k < n; ++k) {
    int oob;
    interp2_bicubic_pre(Z, DX, DY, DXY, H, W, XI[k], YI[k], &ZI[k], &ZXI[k], &ZYI[k], &oob);
  }
  free(DX); free(DY); free(DXY);
}

/* cubic B-spline prefilter, mirror boundary (scipy.ndimage.spline_filter,
 * which map_coordinates(order=3, mode='constant') applies; derivatives.py:244-283) */
static void bspline_filter1d(double *c, long n, long stride) {
  if (n == 1) return;
  const double z = sqrt(3.0) - 2.0, gain = (1 - z) * (1 - 1 / z);
  for (long i = 0; i < n; ++i) c[i * stride] *= gain;
  /* causal init for a whole-sample mirrored signal */
  double zn = pow(z, (double)(n - 1)), zi = z;
  double c0 = c[0] + zn * c[(n - 1) * stride];
  for (long i = 1; i < n - 1; ++i) { c0 += zi * (c[i * stride] + zn * c[(n - 1 - i) * stride]); zi *= z; }
  c[0] = c0 / (1 - zn * zn);
  for (long i = 1; i < n; ++i) c[i * stride] += z * c[(i - 1) * stride];
  c[(n - 1) * stride] = (z * c[(n - 2) * stride] + c[(n - 1) * stride]) * z / (z * z - 1);
  for (long i = n - 2; i >= 0; --i) c[i * stride] = z * (c[(i + 1) * stride] - c[i * stride]);
}
void ofr_bspline_prefilter(const double *in, int H, int W, double *out) {
  memcpy(out, in, (long)H * W * sizeof(double));
  for (int i = 0; i < H; ++i) bspline_filter1d(out + (long)i * W, W, 1);
  for (int j = 0; j < W; ++j) bspline_filter1d(out + j, H, W);
}
static inline double bspline3(double t) {
  t = fabs(t);
  if (t < 1) return 2.0 / 3.0 - t * t + 0.5 * t * t * t;
  if (t < 2) { double s = 2 - t; return s * s * s / 6.0; }
  return 0.0;
}
/* map_coordinates(order=3, mode='constant', cval=nan) on prefiltered coefs, 0-based */
static double bspline_eval(const double *c, int H, int W, double r, double q) {
  if (!(r >= 0 && r <= H - 1 && q >= 0 && q <= W - 1)) return NAN;
  int i0 = (int)floor(r), j0 = (int)floor(q);
  double s = 0;
  for (int a = -1; a <= 2; ++a) {
    double wr = bspline3(r - (i0 + a));
    int ii = ext_mirror(i0 + a, H);
    double t = 0;
    for (int b = -1; b <= 2; ++b) t += bspline3(q - (j0 + b)) * c[IDX(ii, ext_mirror(j0 + b, W), W)];
    s += wr * t;
  }
  return s;
}
/* map_coordinates(order=1, mode='constant', cval=nan), 0-based */
static double bilinear_eval_nan(const double *a, int H, int W, double r, double q) {
  if (!(r >= 0 && r <= H - 1 && q >= 0 && q <= W - 1)) return NAN;
  return bilin_clamped(a, H, W, r, q);
}

/* partial_deriv (derivatives.py:148-296).  images planar 2*nc, uv planar 2,
 * outputs planar nc. */
void ofr_partial_deriv(const double *images, int H, int W, int nc, const double *uv, int interp,
                       const double *filt, double blend, double *It, double *Ix, double *Iy) {
  long N = (long)H * W;
  double *I1x = malloc(N * sizeof(double)), *I1y = malloc(N * sizeof(double));
  double *A = malloc(N * sizeof(double)), *B = malloc(N * sizeof(double)), *Cc = malloc(N * sizeof(double));
  double *Ab = malloc(N * sizeof(double)), *Bb = malloc(N * sizeof(double)), *Cb = malloc(N * sizeof(double));
  for (int ch = 0; ch < nc; ++ch) {
    const double *im1 = images + (long)ch * N, *im2 = images + (long)(nc + ch) * N;
    ofr_deriv_grids(im1, H, W, filt, I1x, I1y, NULL);
    double *it = It + (long)ch * N, *ix = Ix + (long)ch * N, *iy = Iy + (long)ch * N;
    if (interp == OF_INTERP_BICUBIC) {
      ofr_deriv_grids(im2, H, W, filt, A, B, Cc); /* DX, DY, DXY of im2 */
#pragma omp parallel for schedule(static) if ((long)H * W > 40000)
      for (int i = 0; i < H; ++i)
        for (int j = 0; j < W; ++j) {
          long k = IDX(i, j, W);
          double x2 = (j + 1) + uv[k], y2 = (i + 1) + uv[N + k];
          double zi, zx, zy;
          int oob;
          interp2_bicubic_pre(im2, A, B, Cc, H, W, x2, y2, &zi, &zx, &zy, &oob);
          if (isnan(zi)) { it[k] = 0; ix[k] = 0; iy[k] = 0; continue; }
          it[k] = zi - im1[k];
          ix[k] = blend * zx + (1 - blend) * I1x[k];
          iy[k] = blend * zy + (1 - blend) * I1y[k];
        }
    } else {
      ofr_deriv_grids(im2, H, W, filt, B, Cc, NULL); /* I2x, I2y */
      if (interp == OF_INTERP_CUBIC) {
        ofr_bspline_prefilter(im2, H, W, Ab);
        ofr_bspline_prefilter(B, H, W, Bb);
        ofr_bspline_prefilter(Cc, H, W, Cb);
      } else {
        memcpy(Ab, im2, N * sizeof(double)); memcpy(Bb, B, N * sizeof(double)); memcpy(Cb, Cc, N * sizeof(double));
      }
#pragma omp parallel for schedule(static) if ((long)H * W > 40000)
      for (int i = 0; i < H; ++i)
        for (int j = 0; j < W; ++j) {
          long k = IDX(i, j, W);
          double x2 = (j + 1) + uv[k], y2 = (i + 1) + uv[N + k];
          int out = (x2 > W) || (x2 < 1) || (y2 > H) || (y2 < 1);
          if (out) { it[k] = 0; ix[k] = 0; iy[k] = 0; continue; }
          double r = y2 - 1, q = x2 - 1, w, wx, wy;
          if (interp == OF_INTERP_CUBIC) {
            w = bspline_eval(Ab, H, W, r, q); wx = bspline_eval(Bb, H, W, r, q); wy = bspline_eval(Cb, H, W, r, q);
          } else {
            w = bilinear_eval_nan(Ab, H, W, r, q); wx = bilinear_eval_nan(Bb, H, W, r, q); wy = bilinear_eval_nan(Cb, H, W, r, q);
          }
          it[k] = w - im1[k];
          ix[k] = blend * wx + (1 - blend) * I1x[k];
          iy[k] = blend * wy + (1 - blend) * I1y[k];
        }
    }
  }
  free(I1x); free(I1y); free(A); free(B); free(Cc); free(Ab); free(Bb); free(Cb);
}

/* ------------------------------------------------------------------ */
/* flow operator: classic_nl.py:279-378, ba.py:208-302, hs.py:144-203  */
/* ------------------------------------------------------------------ */
/* Matrix-free form of A = [[diag(psi Ix2)+lam FU, diag(psi Ixy)], [.., diag(psi Iy2)+lam FV]]
 * where FU = Dx' diag(wx) Dx + Dy' diag(wy) Dy is a weighted 5-point graph
 * Laplacian (make_convn_mat 'valid'+'sameswap': Dx u(i,j) = u(i,j+1)-u(i,j),
 * zero at j=W-1; sparse_ops.py:59-110).  coef planes:
 *   0 wx_u (edge (i,j)-(i,j+1)), 1 wy_u (edge (i,j)-(i+1,j)), 2 wx_v, 3 wy_v,
 *   4 a_uu, 5 a_uv, 6 a_vv;  rhs planes 0 b_u, 1 b_v.
 * GNC blend A = alpha A_q + (1-alpha) A_r (classic_nl.py:237-248) is applied
 * per coefficient.  Optional AltBA coupling (alt_ba.py:236-242). */
void ofr_flow_operator_ex(const of_params *P, double alpha, const double *uv, const double *duv,
                          const double *It, const double *Ix, const double *Iy, int H, int W, int nc,
                          const double *uvhat, double lambda2, double *coef, double *rhs) {
  long N = (long)H * W;
  int use_q = alpha > 0, use_r = alpha < 1;
  double aq = use_r ? alpha : 1.0, ar = use_q ? 1.0 - alpha : 1.0;
  double lq = P->lambda_q, lr = P->lambda_;
  double *wx_u = coef, *wy_u = coef + N, *wx_v = coef + 2 * N, *wy_v = coef + 3 * N;
#pragma omp parallel for schedule(static) if ((long)H * W > 40000)
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) {
      long k = IDX(i, j, W);
      double u = uv[k] + (duv ? duv[k] : 0), v = uv[N + k] + (duv ? duv[N + k] : 0);
      double wxu = 0, wyu = 0, wxv = 0, wyv = 0;
      if (j < W - 1) {
        double du = uv[k + 1] + (duv ? duv[k + 1] : 0) - u, dv = uv[N + k + 1] + (duv ? duv[N + k + 1] : 0) - v;
        if (use_q) { wxu += aq * lq * pen_w(&P->qua_spatial_u[0], du); wxv += aq * lq * pen_w(&P->qua_spatial_v[0], dv); }
        if (use_r) { wxu += ar * lr * pen_w(&P->rho_spatial_u[0], du); wxv += ar * lr * pen_w(&P->rho_spatial_v[0], dv); }
      }
      if (i < H - 1) {
        double du = uv[k + W] + (duv ? duv[k + W] : 0) - u, dv = uv[N + k + W] + (duv ? duv[N + k + W] : 0) - v;
        if (use_q) { wyu += aq * lq * pen_w(&P->qua_spatial_u[1], du); wyv += aq * lq * pen_w(&P->qua_spatial_v[1], dv); }
        if (use_r) { wyu += ar * lr * pen_w(&P->rho_spatial_u[1], du); wyv += ar * lr * pen_w(&P->rho_spatial_v[1], dv); }
      }
      wx_u[k] = wxu; wy_u[k] = wyu; wx_v[k] = wxv; wy_v[k] = wyv;
    }
#pragma omp parallel for schedule(static) if ((long)H * W > 40000)
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) {
      long k = IDX(i, j, W);
      /* data term, channel-averaged as in classic_nl.py:330-343 */
      double du = duv ? duv[k] : 0, dv = duv ? duv[N + k] : 0;
      double psi_q = 0, psi_r = 0, ix2 = 0, iy2 = 0, ixy = 0, itx = 0, ity = 0;
      for (int c = 0; c < nc; ++c) {
        long kc = (long)c * N + k;
        double itl = It[kc] + Ix[kc] * du + Iy[kc] * dv;
        if (use_q) psi_q += pen_w(&P->qua_data, itl);
        if (use_r) psi_r += pen_w(&P->rho_data, itl);
        ix2 += Ix[kc] * Ix[kc]; iy2 += Iy[kc] * Iy[kc]; ixy += Ix[kc] * Iy[kc];
        itx += itl * Ix[kc]; ity += itl * Iy[kc];
      }
      psi_q /= nc; psi_r /= nc; ix2 /= nc; iy2 /= nc; ixy /= nc; itx /= nc; ity /= nc;
      double psi = (use_q ? aq * psi_q : 0) + (use_r ? ar * psi_r : 0);
      double eL = j > 0 ? wx_u[k - 1] : 0, eR = wx_u[k], eU = i > 0 ? wy_u[k - W] : 0, eD = wy_u[k];
      double fL = j > 0 ? wx_v[k - 1] : 0, fR = wx_v[k], fU = i > 0 ? wy_v[k - W] : 0, fD = wy_v[k];
      double uc = uv[k], vc = uv[N + k];
      double lu = eR * (uc - (j < W - 1 ? uv[k + 1] : 0)) + eD * (uc - (i < H - 1 ? uv[k + W] : 0)) +
                  eL * (uc - (j > 0 ? uv[k - 1] : 0)) + eU * (uc - (i > 0 ? uv[k - W] : 0));
      double lv = fR * (vc - (j < W - 1 ? uv[N + k + 1] : 0)) + fD * (vc - (i < H - 1 ? uv[N + k + W] : 0)) +
                  fL * (vc - (j > 0 ? uv[N + k - 1] : 0)) + fU * (vc - (i > 0 ? uv[N + k - W] : 0));
      double auu = psi * ix2 + (eL + eR + eU + eD), avv = psi * iy2 + (fL + fR + fU + fD);
      double bu = -lu - psi * itx, bv = -lv - psi * ity;
      if (uvhat) {
        double tu = pen_w(&P->rho_couple, uv[k] - uvhat[k]), tv = pen_w(&P->rho_couple, uv[N + k] - uvhat[N + k]);
        auu += lambda2 * tu; avv += lambda2 * tv;
        bu += lambda2 * tu * (uvhat[k] - uv[k]);
        bv += lambda2 * tv * (uvhat[N + k] - uv[N + k]);
      }
      coef[4 * N + k] = auu; coef[5 * N + k] = psi * ixy; coef[6 * N + k] = avv;
      rhs[k] = bu; rhs[N + k] = bv;
    }
}
void ofr_flow_operator(const of_params *P, double alpha, const double *uv, const double *duv, const double *It,
                       const double *Ix, const double *Iy, int H, int W, int nc, double *coef, double *rhs) {
  ofr_flow_operator_ex(P, alpha, uv, duv, It, Ix, Iy, H, W, nc, NULL, 0.0, coef, rhs);
}

/* y = A x on the matrix-free operator; x, y planar (u plane, v plane) */
static void op_apply(const double *coef, int H, int W, const double *x, double *y) {
  long N = (long)H * W;
  const double *wxu = coef, *wyu = coef + N, *wxv = coef + 2 * N, *wyv = coef + 3 * N;
#pragma omp parallel for schedule(static) if ((long)H * W > 40000)
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) {
      long k = IDX(i, j, W);
      double su = 0, sv = 0;
      if (j < W - 1) { su += wxu[k] * x[k + 1]; sv += wxv[k] * x[N + k + 1]; }
      if (j > 0) { su += wxu[k - 1] * x[k - 1]; sv += wxv[k - 1] * x[N + k - 1]; }
      if (i < H - 1) { su += wyu[k] * x[k + W]; sv += wyv[k] * x[N + k + W]; }
      if (i > 0) { su += wyu[k - W] * x[k - W]; sv += wyv[k - W] * x[N + k - W]; }
      y[k] = coef[4 * N + k] * x[k] + coef[5 * N + k] * x[N + k] - su;
      y[N + k] = coef[5 * N + k] * x[k] + coef[6 * N + k] * x[N + k] - sv;
    }
}
static double dotp(const double *a, const double *b, long n) {
  double s = 0;
  for (long k = 0; k < n; ++k) s += a[k] * b[k];
  return s;
}

/* scipy.sparse.linalg.cg with a Jacobi (block=0) or 2x2-block-Jacobi (block=1)
 * preconditioner, x0 = 0 (base.py:116-136) */
static int pcg(const double *coef, const double *b, int H, int W, double rtol, int maxiter, int block,
               const double *x0, double *x, double *relres) {
  long N = (long)H * W, n2 = 2 * N;
  double *r = malloc(n2 * sizeof(double)), *z = malloc(n2 * sizeof(double));
  double *p = malloc(n2 * sizeof(double)), *q = malloc(n2 * sizeof(double));
  double bn = sqrt(dotp(b, b, n2)), atol = rtol * bn;
  memset(x, 0, n2 * sizeof(double));
  memcpy(r, b, n2 * sizeof(double));
  if (x0) { /* warm start (experiment knob ofr_set_warm_start): r = b - A x0 */
    memcpy(x, x0, n2 * sizeof(double));
    op_apply(coef, H, W, x0, q);
    for (long k = 0; k < n2; ++k) r[k] = b[k] - q[k];
  }
  int it = 0;
  double rho_prev = 0;
  if (bn == 0) { *relres = 0; free(r); free(z); free(p); free(q); return 0; }
  for (it = 0; it < maxiter; ++it) {
    if (sqrt(dotp(r, r, n2)) < atol) break;
    for (long k = 0; k < N; ++k) {
      double a = coef[4 * N + k], c = coef[5 * N + k], d = coef[6 * N + k];
      if (block) {
        double det = a * d - c * c;
        z[k] = (d * r[k] - c * r[N + k]) / det;
        z[N + k] = (a * r[N + k] - c * r[k]) / det;
      } else {
        z[k] = fabs(a) > 1e-12 ? r[k] / a : 0.0;
        z[N + k] = fabs(d) > 1e-12 ? r[N + k] / d : 0.0;
      }
    }
    double rho = dotp(r, z, n2);
    if (it > 0) { double beta = rho / rho_prev; for (long k = 0; k < n2; ++k) p[k] = z[k] + beta * p[k]; }
    else memcpy(p, z, n2 * sizeof(double));
    op_apply(coef, H, W, p, q);
    double alpha = rho / dotp(p, q, n2);
    for (long k = 0; k < n2; ++k) { x[k] += alpha * p[k]; r[k] -= alpha * q[k]; }
    rho_prev = rho;
  }
  *relres = sqrt(dotp(r, r, n2)) / bn;
  free(r); free(z); free(p); free(q);
  return it;
}

/* _sor_solve (base.py:138-172): lexicographic scalar SOR over the
 * column-major [u; v] unknown vector, x0 = 0 */
static int sor(const double *coef, const double *b, int H, int W, double omega, int maxit, double tol,
               double *x) {
  long N = (long)H * W, n2 = 2 * N;
  double *xo = malloc(n2 * sizeof(double));
  memset(x, 0, n2 * sizeof(double));
  int it;
  for (it = 0; it < maxit; ++it) {
    memcpy(xo, x, n2 * sizeof(double));
    for (int comp = 0; comp < 2; ++comp)
      for (int j = 0; j < W; ++j)
        for (int i = 0; i < H; ++i) {
          long k = IDX(i, j, W), row = comp * N + k;
          const double *wx = coef + (comp ? 2 : 0) * N, *wy = coef + (comp ? 3 : 1) * N;
          double diag = coef[(comp ? 6 : 4) * N + k];
          if (fabs(diag) < 1e-15) continue;
          double s = diag * x[row] + coef[5 * N + k] * x[(1 - comp) * N + k];
          if (j < W - 1) s -= wx[k] * x[row + 1];
          if (j > 0) s -= wx[k - 1] * x[row - 1];
          if (i < H - 1) s -= wy[k] * x[row + W];
          if (i > 0) s -= wy[k - W] * x[row - W];
          double sigma = s - diag * x[row];
          x[row] = (1 - omega) * x[row] + omega * (b[row] - sigma) / diag;
        }
    double dn = 0, xn = 0;
    for (long k = 0; k < n2; ++k) { dn += (x[k] - xo[k]) * (x[k] - xo[k]); xn += x[k] * x[k]; }
    if (sqrt(dn) < tol * sqrt(xn)) { ++it; break; }
  }
  free(xo);
  return it;
}

/* _solve_linear_system (base.py:87-114).  'backslash' (SuperLU) is restated as
 * a PCG solve to rtol 1e-12 (fp64), i.e. the direct solution to ~1e-10.
 * ofr_set_backslash_rtol (test-only experiment knob, tools/rtol_chaos.py):
 * another stopping tolerance for that PCG, to separate the GPU surrogate's
 * rtol from fp32 arithmetic; <= 0 restores 1e-12. */
static double g_backslash_rtol = 1e-12;
void ofr_set_backslash_rtol(double rtol) { g_backslash_rtol = rtol > 0 ? rtol : 1e-12; }
/* ofr_set_round_x_f32 (test-only experiment knob, tools/rtol_chaos.py): round
 * every 'backslash' solution to float32, as the GPU returns it, to measure
 * what fp32 storage of x alone does to the chaotic family. */
static int g_round_x_f32 = 0;
void ofr_set_round_x_f32(int on) { g_round_x_f32 = on != 0; }
/* ofr_set_warm_start (test-only experiment knob, tools/warm_start_iters.py):
 * the starting iterate of the 'backslash' PCG in irls_base's warps after the
 * first of a level (the reference's spsolve takes none, base.py:107-108, so
 * its answer does not depend on it; only the iteration count does).
 *   0  x0 = 0 (the default)
 *   1  the previous warp's unclipped solution
 *   2  (uv_prev + x_prev, before the filter) - uv: the part of the previous
 *      step the median filter took back
 *   +10  the same direction scaled by gamma = x0.b / x0.A x0 (the A-norm
 *        optimal multiple; gamma x0 is never worse than 0 in the A-norm)
 * ofr_solve_log: per solve (H, W, warp index, iterations, 1000 * alpha) */
static int g_warm = 0;
static const double *g_x0 = NULL;
void ofr_set_warm_start(int mode) { g_warm = mode; }
#define OFR_SLOG_MAX 4096
static int g_slog[OFR_SLOG_MAX][5];
static int g_slog_n = 0;
int ofr_solve_log(int *out, int max) {
  int n = g_slog_n < max ? g_slog_n : max;
  if (out) memcpy(out, g_slog, (size_t)n * 5 * sizeof(int));
  g_slog_n = 0;
  return n;
}

int ofr_solve(const of_params *P, const double *coef, const double *rhs, int H, int W, double *x, int *iters,
              double *relres) {
  double rr = 0;
  int it;
  if (P->solver == OF_SOLVER_PCG) it = pcg(coef, rhs, H, W, P->pcg_rtol, P->pcg_maxiter, 0, NULL, x, &rr);
  else if (P->solver == OF_SOLVER_SOR) it = sor(coef, rhs, H, W, 1.9, P->sor_max_iters, 1e-2, x);
  else {
    it = pcg(coef, rhs, H, W, g_backslash_rtol, 100000, 1, g_x0, x, &rr);
    if (g_round_x_f32)
      for (long k = 0; k < 2L * H * W; ++k) x[k] = (double)(float)x[k];
  }
  if (iters) *iters = it;
  if (relres) *relres = rr;
  return 0;
}

/* ------------------------------------------------------------------ */
/* occlusion + filters: occlusion.py:6-56, weighted_median.py:5-112     */
/* ------------------------------------------------------------------ */
void ofr_detect_occlusion(const double *uv, const double *images, int H, int W, int nc, double *occ) {
  long N = (long)H * W;
  const double sd = 0.3, si = 20.0;
#pragma omp parallel for schedule(static) if ((long)H * W > 40000)
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) {
      long k = IDX(i, j, W);
      double dudx = j > 0 ? uv[k] - uv[k - 1] : 0.0, dvdy = i > 0 ? uv[N + k] - uv[N + k - W] : 0.0;
      double div = dudx + dvdy;
      double odiv = exp(-div * div / (2 * sd * sd));
      double r = i + uv[N + k], q = j + uv[k];
      r = r < 0 ? 0 : (r > H - 1 ? H - 1 : r);
      q = q < 0 ? 0 : (q > W - 1 ? W - 1 : q);
      double it = 0;
      for (int c = 0; c < nc; ++c)
        it += fabs(bilin_clamped(images + (long)(nc + c) * N, H, W, r, q) - images[(long)c * N + k]);
      if (nc > 1) it /= nc;
      occ[k] = odiv * exp(-it * it / (2 * si * si));
    }
}

typedef struct { double v, w; } vw_t;
static int cmp_vw(const void *a, const void *b) {
  double x = ((const vw_t *)a)->v, y = ((const vw_t *)b)->v;
  return (x > y) - (x < y);
}
/* weighted_median_1d (weighted_median.py:5-21) */
static double wmedian(vw_t *s, int n) {
  qsort(s, n, sizeof(vw_t), cmp_vw);
  double cum = 0, *cw = malloc(n * sizeof(double));
  for (int t = 0; t < n; ++t) { cum += s[t].w; cw[t] = cum; }
  double half = cw[n - 1] / 2.0;
  int idx = n - 1;
  for (int t = 0; t < n; ++t) if (cw[t] >= half) { idx = t; break; }
  free(cw);
  return s[idx].v;
}

/* denoise_color_weighted_medfilt2 / _wmedfilt_vectorized (weighted_median.py:24-112);
 * guide planar gc x H x W; guide == NULL -> 5x5 median fallback (:42-47) */
void ofr_median_filter(const double *in, int H, int W, int planes, int size, double *out);
void ofr_weighted_median(const double *uv, const double *guide, int gc, const double *occ, int H, int W,
                         int hsz, double sigma_i, int mfsz, double *out) {
  long N = (long)H * W;
  if (!guide) { ofr_median_filter(uv, H, W, 2, mfsz, out); return; }
  const double inv = 1.0 / (2.0 * sigma_i * sigma_i);
  int n = (2 * hsz + 1) * (2 * hsz + 1);
#pragma omp parallel if ((long)H * W > 40000)
  {
    vw_t *su = malloc(n * sizeof(vw_t)), *sv = malloc(n * sizeof(vw_t));
#pragma omp for schedule(static)
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < W; ++j) {
        int t = 0;
        for (int a = -hsz; a <= hsz; ++a) {
          int ii = ext_mirror(i + a, H);
          for (int b = -hsz; b <= hsz; ++b, ++t) {
            long q = IDX(ii, ext_mirror(j + b, W), W);
            double d = 0;
            for (int c = 0; c < gc; ++c) {
              double e = guide[(long)c * N + q] - guide[(long)c * N + IDX(i, j, W)];
              d += e * e;
            }
            double w = exp(-d * inv) * occ[q];
            w = w > 1e-10 ? w : 1e-10;
            su[t].v = uv[q]; su[t].w = w;
            sv[t].v = uv[N + q]; sv[t].w = w;
          }
        }
        out[IDX(i, j, W)] = wmedian(su, n);
        out[N + IDX(i, j, W)] = wmedian(sv, n);
      }
    free(su); free(sv);
  }
}

static int cmp_d(const void *a, const void *b) {
  double x = *(const double *)a, y = *(const double *)b;
  return (x > y) - (x < y);
}
/* scipy.ndimage.median_filter(size, mode='reflect') per plane (hs.py:96-97, ba.py:198-199) */
void ofr_median_filter(const double *in, int H, int W, int planes, int size, double *out) {
  int h = size / 2, n = size * size;
  for (int c = 0; c < planes; ++c) {
    const double *a = in + (long)c * H * W;
    double *o = out + (long)c * H * W;
#pragma omp parallel if ((long)H * W > 40000)
    {
      double *buf = malloc(n * sizeof(double));
#pragma omp for schedule(static)
      for (int i = 0; i < H; ++i)
        for (int j = 0; j < W; ++j) {
          int t = 0;
          for (int x = -h; x <= h; ++x)
            for (int y = -h; y <= h; ++y) buf[t++] = a[IDX(ext_reflect(i + x, H), ext_reflect(j + y, W), W)];
          qsort(buf, n, sizeof(double), cmp_d);
          o[IDX(i, j, W)] = buf[n / 2];
        }
      free(buf);
    }
  }
}

/* ------------------------------------------------------------------ */
/* drivers: hs.py:49-142, ba.py:57-204, classic_nl.py:89-277,          */
/*          alt_ba.py:81-274                                            */
/* ------------------------------------------------------------------ */
typedef struct { int H, W; double *im; double *guide; } level_t;

static int build_pyramid(const double *im, int H, int W, int C, int levels, double spacing, level_t *out,
                         int guide_slot) {
  /* _build_pyramid (base.py:174-190): sigma = sqrt(spacing)/sqrt(2), size 2*round(1.5 sigma)+1 */
  double sig = sqrt(spacing) / sqrt(2.0);
  int ks = 2 * (int)nearbyint(1.5 * sig) + 1;
  double *k = malloc(ks * ks * sizeof(double));
  ofr_gaussian(ks, sig, k);
  int n = levels < 1 ? 1 : levels;
  int h = H, w = W;
  double *cur = malloc((long)C * H * W * sizeof(double));
  memcpy(cur, im, (long)C * H * W * sizeof(double));
  for (int l = 0; l < n; ++l) {
    if (l > 0) {
      int nh, nw;
      ofr_resize_dims(h, w, 1.0 / spacing, &nh, &nw);
      double *nx = malloc((long)C * nh * nw * sizeof(double));
      ofr_pyramid_level(cur, h, w, C, k, ks, 1.0 / spacing, nx, &nh, &nw);
      cur = nx;
      h = nh; w = nw;
    }
    out[l].H = h; out[l].W = w;
    if (guide_slot) out[l].guide = cur; else out[l].im = cur;
  }
  free(k);
  return n;
}

static int auto_levels(int H, int W, double spacing) {
  int m = H < W ? H : W; /* base.py:192-195 */
  return 1 + (int)floor(log(m / 16.0) / log(spacing));
}

static void clip_update(double *x, long n) {
  for (long k = 0; k < n; ++k) x[k] = x[k] < -1 ? -1 : (x[k] > 1 ? 1 : x[k]);
}

typedef struct {
  const of_params *P;
  of_stats *st;
  int nc, gc;
} drv_t;

static void note_solve(drv_t *d, int it) {
  if (!d->st) return;
  d->st->solves++;
  d->st->solver_iters_total += it;
  if (it > d->st->solver_iters_max) d->st->solver_iters_max = it;
}

/* HSOpticalFlow.compute_flow_base (hs.py:109-142) */
static void hs_base(drv_t *d, const level_t *L, double *uv) {
  const of_params *P = d->P;
  int H = L->H, W = L->W, nc = d->nc;
  long N = (long)H * W;
  double *It = malloc(nc * N * sizeof(double)), *Ix = malloc(nc * N * sizeof(double)), *Iy = malloc(nc * N * sizeof(double));
  double *coef = malloc(7 * N * sizeof(double)), *rhs = malloc(2 * N * sizeof(double)), *x = malloc(2 * N * sizeof(double));
  double *tmp = malloc(2 * N * sizeof(double));
  for (int i = 0; i < P->max_warping_iters; ++i) {
    ofr_partial_deriv(L->im, H, W, nc, uv, P->interp, P->deriv_filter, 0.5, It, Ix, Iy);
    ofr_flow_operator(P, 0.0, uv, NULL, It, Ix, Iy, H, W, nc, coef, rhs);
    int it;
    ofr_solve(P, coef, rhs, H, W, x, &it, NULL);
    note_solve(d, it);
    if (sqrt(dotp(x, x, 2 * N)) < 1e-3) break;
    if (P->limit_update) clip_update(x, 2 * N);
    for (long k = 0; k < 2 * N; ++k) uv[k] += x[k];
    if (P->median_filter_size)
      for (int m = 0; m < P->mf_iter; ++m) {
        ofr_median_filter(uv, H, W, 2, P->median_filter_size, tmp);
        memcpy(uv, tmp, 2 * N * sizeof(double));
      }
  }
  free(It); free(Ix); free(Iy); free(coef); free(rhs); free(x); free(tmp);
}

/* BAOpticalFlow / ClassicNLOpticalFlow compute_flow_base (ba.py:162-204,
 * classic_nl.py:200-277) */
static void irls_base(drv_t *d, const level_t *L, double *uv, double alpha, int max_linear) {
  const of_params *P = d->P;
  int H = L->H, W = L->W, nc = d->nc;
  long N = (long)H * W;
  double *It = malloc(nc * N * sizeof(double)), *Ix = malloc(nc * N * sizeof(double)), *Iy = malloc(nc * N * sizeof(double));
  double *coef = malloc(7 * N * sizeof(double)), *rhs = malloc(2 * N * sizeof(double)), *x = malloc(2 * N * sizeof(double));
  double *duv = malloc(2 * N * sizeof(double)), *uv1 = malloc(2 * N * sizeof(double)), *occ = malloc(N * sizeof(double));
  double *tmp = malloc(2 * N * sizeof(double));
  double *xw = malloc(2 * N * sizeof(double)), *xp = malloc(2 * N * sizeof(double));
  double *upre = malloc(2 * N * sizeof(double));
  double blend = P->method == OF_METHOD_BA ? P->blend : 0.5; /* classic_nl.py:232 passes no blend */
  for (int i = 0; i < P->max_iters; ++i) {
    memset(duv, 0, 2 * N * sizeof(double));
    ofr_partial_deriv(L->im, H, W, nc, uv, P->interp, P->deriv_filter, blend, It, Ix, Iy);
    for (int j = 0; j < max_linear; ++j) {
      ofr_flow_operator(P, alpha, uv, duv, It, Ix, Iy, H, W, nc, coef, rhs);
      int it;
      g_x0 = NULL;
      if (g_warm % 10 && i > 0 && j == 0) {
        for (long k = 0; k < 2 * N; ++k) xw[k] = g_warm % 10 == 1 ? xp[k] : upre[k] - uv[k];
        if (g_warm >= 10) {
          op_apply(coef, H, W, xw, tmp);
          double xAx = dotp(xw, tmp, 2 * N), xb = dotp(xw, rhs, 2 * N), gam = xAx > 0 ? xb / xAx : 0.0;
          for (long k = 0; k < 2 * N; ++k) xw[k] *= gam;
        }
        g_x0 = xw;
      }
      ofr_solve(P, coef, rhs, H, W, x, &it, NULL);
      g_x0 = NULL;
      note_solve(d, it);
      if (g_slog_n < OFR_SLOG_MAX) {
        int *e = g_slog[g_slog_n++];
        e[0] = H; e[1] = W; e[2] = i; e[3] = it; e[4] = (int)lround(alpha * 1000);
      }
      memcpy(xp, x, 2 * N * sizeof(double));
      for (long k = 0; k < 2 * N; ++k) upre[k] = uv[k] + x[k];
      if (P->limit_update) clip_update(x, 2 * N);
      for (long k = 0; k < 2 * N; ++k) uv1[k] = uv[k] + x[k];
      if (P->median_filter_size) {
        if (P->method == OF_METHOD_CLASSIC_NL) {
          ofr_detect_occlusion(uv1, L->im, H, W, nc, occ);
          ofr_weighted_median(uv1, L->guide, d->gc, occ, H, W, P->area_hsz, P->sigma_i, P->median_filter_size, tmp);
        } else {
          ofr_median_filter(uv1, H, W, 2, P->median_filter_size, tmp);
        }
        memcpy(uv1, tmp, 2 * N * sizeof(double));
      }
      for (long k = 0; k < 2 * N; ++k) duv[k] = uv1[k] - uv[k];
    }
    for (long k = 0; k < 2 * N; ++k) uv[k] += duv[k];
  }
  free(It); free(Ix); free(Iy); free(coef); free(rhs); free(x); free(duv); free(uv1); free(occ); free(tmp);
  free(xw); free(xp); free(upre);
}

/* denoise_LO (denoising.py:6-30) */
static void denoise_lo(const double *un, int H, int W, int mfsz, double lam, int iters, double *u) {
  long N = (long)H * W;
  memcpy(u, un, N * sizeof(double));
  if (!mfsz) return;
  double *t = malloc(N * sizeof(double));
  for (int it = 0; it < iters; ++it) {
    for (long k = 0; k < N; ++k) t[k] = u[k] + lam * (un[k] - u[k]);
    ofr_median_filter(t, H, W, 1, mfsz, u);
  }
  free(t);
}

/* AltBAOpticalFlow.compute_flow_base (alt_ba.py:189-274) */
static void altba_base(drv_t *d, const level_t *L, double *uv, double *uvhat, double alpha, int replacement) {
  const of_params *P = d->P;
  int H = L->H, W = L->W, nc = d->nc;
  long N = (long)H * W;
  double *It = malloc(nc * N * sizeof(double)), *Ix = malloc(nc * N * sizeof(double)), *Iy = malloc(nc * N * sizeof(double));
  double *coef = malloc(7 * N * sizeof(double)), *rhs = malloc(2 * N * sizeof(double)), *x = malloc(2 * N * sizeof(double));
  double *duv = malloc(2 * N * sizeof(double));
  int n = P->max_iters;
  double *l2s = malloc((n + 1) * sizeof(double));
  double a = log10(1e-4), b = log10(P->lambda2);
  for (int t = 0; t < n; ++t) l2s[t] = pow(10.0, n == 1 ? a : a + (b - a) * t / (n - 1)); /* np.logspace */
  l2s[n] = P->lambda2;
  double lambda2 = l2s[0];
  for (int i = 0; i < n; ++i) {
    memset(duv, 0, 2 * N * sizeof(double));
    ofr_partial_deriv(L->im, H, W, nc, uv, P->interp, P->deriv_filter, 0.5, It, Ix, Iy);
    for (int j = 0; j < P->max_linear; ++j) {
      ofr_flow_operator_ex(P, alpha, uv, duv, It, Ix, Iy, H, W, nc, uvhat, lambda2, coef, rhs);
      int it;
      ofr_solve(P, coef, rhs, H, W, x, &it, NULL);
      note_solve(d, it);
      if (P->limit_update) clip_update(x, 2 * N);
      memcpy(duv, x, 2 * N * sizeof(double));
    }
    for (long k = 0; k < 2 * N; ++k) uv[k] += duv[k];
    for (int c = 0; c < 2; ++c)
      denoise_lo(uv + c * N, H, W, P->median_filter_size, lambda2 / P->lambda3, P->itersLO, uvhat + c * N);
    if (replacement) memcpy(uv, uvhat, 2 * N * sizeof(double));
    lambda2 = l2s[i + 1];
  }
  free(It); free(Ix); free(Iy); free(coef); free(rhs); free(x); free(duv); free(l2s);
}

/* AltBAOpticalFlow.compute_flow_base(uv, uvhat) on one level (alt_ba.py:189-274);
 * images planar 2*nc, uv and uvhat planar 2 x H x W, updated in place */
void ofr_alt_ba_flow_base(const of_params *P, const double *images, int H, int W, int nc, double alpha,
                          int replacement, double *uv, double *uvhat) {
  drv_t d = {P, NULL, nc, 0};
  level_t L = {H, W, (double *)images, NULL};
  altba_base(&d, &L, uv, uvhat, alpha, replacement);
}

/* compute_flow for all four methods.  images planar 2*nc (frame-1 channels
 * then frame-2 channels); guide planar gc or NULL; init_uv may be NULL.
 * P->alpha is updated to the final GNC alpha (restored for BA). */
int ofr_compute_flow(of_params *P, const double *images, int H, int W, int nc, const double *guide, int gc,
                     const double *init_uv, double *out_uv, of_stats *st) {
  /* the restatement covers the default spatial_filters pair only; general
   * lists are pinned by the reference's own fixtures (tests/golden/filters.npz) */
  if (P->filters.general) return OF_ENOTSUP;
  long N = (long)H * W;
  int C = 2 * nc;
  drv_t d = {P, st, nc, gc};
  if (st) memset(st, 0, sizeof(*st));
  double *uv = malloc(2 * N * sizeof(double));
  if (init_uv) memcpy(uv, init_uv, 2 * N * sizeof(double)); else memset(uv, 0, 2 * N * sizeof(double));
  /* preprocessing (classic_nl.py:106-115, ba.py:277-287, hs.py:66-70, alt_ba.py:100-104) */
  double *img = malloc(C * N * sizeof(double));
  if (P->texture) {
    double alp = (P->method == OF_METHOD_HS || P->method == OF_METHOD_ALT_BA) ? 0.95 : P->alp;
    ofr_rof_texture(images, H, W, C, 1.0 / 8, 100, alp, img);
  } else if (P->fc && (P->method == OF_METHOD_BA || P->method == OF_METHOD_CLASSIC_NL)) {
    double g[25], *t = malloc(N * sizeof(double));
    ofr_gaussian(5, 1.5, g);
    for (int c = 0; c < C; ++c) {
      ofr_correlate(images + c * N, H, W, g, 5, 5, t);
      for (long k = 0; k < N; ++k) img[c * N + k] = images[c * N + k] - P->alp * t[k];
    }
    free(t);
    ofr_scale_image(img, C * N, 0, 255);
  } else {
    memcpy(img, images, C * N * sizeof(double));
    ofr_scale_image(img, C * N, 0, 255);
  }
  int levels = P->pyramid_levels;
  if (P->method == OF_METHOD_HS || P->method == OF_METHOD_ALT_BA || P->auto_level)
    levels = auto_levels(H, W, P->pyramid_spacing);
  P->pyramid_levels = levels;
  level_t pyr[OF_MAX_LEVELS] = {0}, gpyr[OF_MAX_LEVELS] = {0};
  int npyr = build_pyramid(img, H, W, C, levels, P->pyramid_spacing, pyr, 0);
  int ngpyr = 0;
  if (P->method != OF_METHOD_HS) ngpyr = build_pyramid(img, H, W, C, P->gnc_pyramid_levels, P->gnc_pyramid_spacing, gpyr, 0);
  if (P->method == OF_METHOD_CLASSIC_NL && guide) {
    build_pyramid(guide, H, W, gc, levels, P->pyramid_spacing, pyr, 1);
    build_pyramid(guide, H, W, gc, P->gnc_pyramid_levels, P->gnc_pyramid_spacing, gpyr, 1);
  }
  double *uvhat = NULL;
  if (P->method == OF_METHOD_ALT_BA) { uvhat = malloc(2 * N * sizeof(double)); memcpy(uvhat, uv, 2 * N * sizeof(double)); }
  int curH = H, curW = W;
  double alpha_orig = P->alpha;
  int gnc = P->method == OF_METHOD_HS ? 1 : P->gnc_iters;
  for (int ig = 0; ig < gnc; ++ig) {
    int nl = ig == 0 ? levels : P->gnc_pyramid_levels;
    level_t *lv = ig == 0 ? pyr : gpyr;
    for (int l = nl - 1; l >= 0; --l) {
      int h = lv[l].H, w = lv[l].W;
      double *nuv = malloc(2L * h * w * sizeof(double));
      ofr_resample_flow(uv, curH, curW, h, w, nuv);
      free(uv); uv = nuv;
      if (uvhat) {
        double *nh = malloc(2L * h * w * sizeof(double));
        ofr_resample_flow(uvhat, curH, curW, h, w, nh);
        free(uvhat); uvhat = nh;
      }
      curH = h; curW = w;
      if (P->method == OF_METHOD_HS) hs_base(&d, &lv[l], uv);
      else if (P->method == OF_METHOD_ALT_BA) altba_base(&d, &lv[l], uv, uvhat, P->alpha, ig != gnc - 1);
      else irls_base(&d, &lv[l], uv, P->alpha, (P->method == OF_METHOD_BA && ig == 0) ? 1 : (ig == 0 ? 1 : P->max_linear));
      if (st && st->n_levels < OF_MAX_LEVELS) {
        st->level_h[st->n_levels] = h; st->level_w[st->n_levels] = w; st->level_stage[st->n_levels] = ig;
        st->n_levels++;
      }
    }
    if (gnc > 1) { /* GNC alpha schedule (classic_nl.py:180-184, ba.py:329-333) */
      double na = 1.0 - (ig + 1.0) / (gnc - 1.0);
      P->alpha = fmax(0.0, fmin(P->alpha, na));
    }
  }
  if (P->method == OF_METHOD_BA) P->alpha = alpha_orig; /* ba.py:338-339 */
  if (P->method == OF_METHOD_HS && P->median_filter_size) { /* hs.py:94-97 */
    double *t = malloc(2 * N * sizeof(double));
    ofr_median_filter(uv, curH, curW, 2, P->median_filter_size, t);
    memcpy(uv, t, 2 * N * sizeof(double));
    free(t);
  }
  if (curH != H || curW != W) { /* no level processed (tiny image): uv keeps init size */
    memcpy(out_uv, init_uv ? init_uv : uv, 2 * N * sizeof(double));
  } else {
    memcpy(out_uv, P->method == OF_METHOD_ALT_BA ? uvhat : uv, 2 * N * sizeof(double));
  }
  for (int l = 0; l < npyr; ++l) { free(pyr[l].im); free(pyr[l].guide); }
  for (int l = 0; l < ngpyr; ++l) { free(gpyr[l].im); free(gpyr[l].guide); }
  free(uv); free(uvhat); free(img);
  return 0;
}

/* estimate_flow (interface.py:11-71) minus parameter parsing: RGB (C==3,
 * interleaved) or gray (C==1).  guide_mode: 1 = the method has a colour
 * guide (color_images not None, i.e. Classic+NL from load_of_method). */
int ofr_estimate_flow(of_params *P, const double *im1, const double *im2, int H, int W, int C,
                      const double *init_uv, double *out_uv, of_stats *st) {
  long N = (long)H * W;
  double *images = malloc(2 * N * sizeof(double)), *guide = NULL;
  int gc = 0;
  if (C >= 3) {
    ofr_rgb2gray(im1, H, W, images);
    ofr_rgb2gray(im2, H, W, images + N);
  } else {
    memcpy(images, im1, N * sizeof(double));
    memcpy(images + N, im2, N * sizeof(double));
  }
  if (P->guide_mode) {
    if (C >= 3) {
      gc = 3;
      guide = malloc(3 * N * sizeof(double));
      ofr_rgb2lab(im1, H, W, guide);
      for (int c = 0; c < 3; ++c) ofr_scale_image(guide + c * N, N, 0, 255);
    } else {
      gc = 1;
      guide = malloc(N * sizeof(double));
      memcpy(guide, im1, N * sizeof(double));
    }
  }
  int rc = ofr_compute_flow(P, images, H, W, 1, guide, gc, init_uv, out_uv, st);
  free(images); free(guide);
  return rc;
}

int ofr_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
