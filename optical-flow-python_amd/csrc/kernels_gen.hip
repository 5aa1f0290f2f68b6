// kernels_gen.hip — the flow operator and its solvers for a GENERAL
// spatial_filters list (classic_nl.py:301-322, ba.py:228-246,
// alt_ba.py:298-316).  The registry's methods all use the default pair
// [[1, -1]], [[1], [-1]], which runs on the matrix-free 5-point hot path
// (k_flow_operator, k_cgs, k_sor_lex); this file serves any other list of up
// to OF_MAX_FILTERS filters of at most 5 x 5 taps.
//
// Operator: A = [[D_uu + lambda FU, D_uv], [D_uv, D_vv + lambda FV]] with FU =
// sum_i F_i^T diag(w_i) F_i, F_i the reference's make_convn_mat(F_i, sz,
// 'valid', 'sameswap') (utils/sparse_ops.py:59-109): row (vi + oi, vj + oj)
// of the same-size output holds the valid convolution at (vi, vj),
//   (F x)(vi, vj) = sum_{a,b} F[a][b] x(vi + fh-1-a, vj + fw-1-b),
// oi = (fh-1)/2, oj = (fw-1)/2, rows outside the valid range are zero.  The
// product F^T W F couples pixels y and y + (a1 - a2, b1 - b2) through every
// tap pair, so A is stored in DIA form on the dense offset grid of radius D
// (G = (2D+1)^2 planes per component + the u-v coupling plane).
//
// Solvers on the DIA form (base.py:87-172): CG with the scipy control flow
// ('pcg': Jacobi 1/diag, rtol pcg_rtol; 'backslash' surrogate: 2x2 block
// Jacobi, rtol exact_rtol met in the fp64 true residual by iterative
// refinement), and the reference's lexicographic SOR as a column-wavefront
// in one workgroup.  Reductions are fixed-order per-block partials.

#define GEN_MAXD (OF_MAX_FDIM - 1)
#define GEN_MAXG ((2 * GEN_MAXD + 1) * (2 * GEN_MAXD + 1))
#define GEN_NT 25

struct GenFilters {
  int n, D;
  int fh[OF_MAX_FILTERS], fw[OF_MAX_FILTERS];
  float taps[OF_MAX_FILTERS][GEN_NT];
  PenF ru[OF_MAX_FILTERS], rv[OF_MAX_FILTERS], qu[OF_MAX_FILTERS], qv[OF_MAX_FILTERS];
};

// per-filter weights w_i (lambda and the GNC blend folded in) at every row
// of the same-size output: 2 n planes (u of filter i at plane 2i, v at 2i+1)
__global__ __launch_bounds__(OF_BX *OF_BY) void k_gen_weights(GenFilters f, OpArgs o, const float2 *__restrict__ uv,
                                                               const float2 *__restrict__ duv, int H, int W, int P,
                                                               size_t ps, float *__restrict__ wpl) {
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    for (int q = 0; q < f.n; ++q) {
      const int fh = f.fh[q], fw = f.fw[q];
      const int vi = i - (fh - 1) / 2, vj = j - (fw - 1) / 2;
      float wu = 0.f, wv = 0.f;
      if (vi >= 0 && vj >= 0 && vi < H - fh + 1 && vj < W - fw + 1) {
        float su = 0.f, sv = 0.f;
        for (int a = 0; a < fh; ++a)
          for (int b = 0; b < fw; ++b) {
            const float t = f.taps[q][a * fw + b];
            const size_t kk = (size_t)(vi + fh - 1 - a) * P + (vj + fw - 1 - b);
            float2 x = uv[kk];
            if (duv) { const float2 d = duv[kk]; x.x += d.x; x.y += d.y; }
            su += t * x.x;
            sv += t * x.y;
          }
        if (o.use_q) { wu += o.aq_s * pen_w(f.qu[q], su); wv += o.aq_s * pen_w(f.qv[q], sv); }
        if (o.use_r) { wu += o.ar_s * pen_w(f.ru[q], su); wv += o.ar_s * pen_w(f.rv[q], sv); }
      }
      wpl[(size_t)(2 * q) * ps + k] = wu;
      wpl[(size_t)(2 * q + 1) * ps + k] = wv;
    }
  }
}

// DIA planes + rhs: offset index e = (di + D) (2D+1) + (dj + D); planes
// [0, G) u-u, [G, 2G) v-v, 2G the u-v coupling
__global__ __launch_bounds__(OF_BX *OF_BY) void k_gen_dia(GenFilters f, OpArgs o, const float *__restrict__ wpl,
                                                           const float2 *__restrict__ uv, const float2 *__restrict__ duv,
                                                           const float *__restrict__ It, const float *__restrict__ Ix,
                                                           const float *__restrict__ Iy, int nc,
                                                           const float2 *__restrict__ uvhat, int H, int W, int P,
                                                           size_t ps, float *__restrict__ pl, float2 *__restrict__ rhs) {
  const int D = f.D, S = 2 * D + 1, G = S * S;
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    // data term, channel-averaged (as k_flow_operator, classic_nl.py:330-343)
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
    float bu = -psi * itx, bv = -psi * ity;
    float d0u = psi * ix2, d0v = psi * iy2;
    if (uvhat) {  // AltBA coupling (alt_ba.py:236-242)
      const float2 u0 = uv[k], h = uvhat[k];
      const float tu = pen_w(o.rc, u0.x - h.x), tv = pen_w(o.rc, u0.y - h.y);
      d0u += o.lambda2 * tu;
      d0v += o.lambda2 * tv;
      bu += o.lambda2 * tu * (h.x - u0.x);
      bv += o.lambda2 * tv * (h.y - u0.y);
    }
    for (int di = -D; di <= D; ++di)
      for (int dj = -D; dj <= D; ++dj) {
        float cu = 0.f, cv = 0.f;
        // tap pairs (a1, b1), (a2, b2) = (a1 - di, b1 - dj) of every filter:
        // row r at valid (vi, vj) = (i - (fh-1-a1), j - (fw-1-b1))
        for (int q = 0; q < f.n; ++q) {
          const int fh = f.fh[q], fw = f.fw[q];
          for (int a1 = max(0, di); a1 < min(fh, fh + di); ++a1)
            for (int b1 = max(0, dj); b1 < min(fw, fw + dj); ++b1) {
              const int vi = i - (fh - 1 - a1), vj = j - (fw - 1 - b1);
              if (vi < 0 || vj < 0 || vi >= H - fh + 1 || vj >= W - fw + 1) continue;
              const float tt = f.taps[q][a1 * fw + b1] * f.taps[q][(a1 - di) * fw + (b1 - dj)];
              const size_t kr = (size_t)(vi + (fh - 1) / 2) * P + (vj + (fw - 1) / 2);
              cu += tt * wpl[(size_t)(2 * q) * ps + kr];
              cv += tt * wpl[(size_t)(2 * q + 1) * ps + kr];
            }
        }
        // b: minus the spatial part of row y times uv (-lambda FU u); the
        // data diagonal does not multiply uv
        const int ii = i + di, jj = j + dj;
        if (ii >= 0 && jj >= 0 && ii < H && jj < W && (cu != 0.f || cv != 0.f)) {
          const float2 n = uv[(size_t)ii * P + jj];
          bu -= cu * n.x;
          bv -= cv * n.y;
        }
        if (di == 0 && dj == 0) {
          cu += d0u;
          cv += d0v;
        }
        const int e = (di + D) * S + (dj + D);
        pl[(size_t)e * ps + k] = cu;
        pl[(size_t)(G + e) * ps + k] = cv;
      }
    pl[(size_t)(2 * G) * ps + k] = psi * ixy;
    rhs[k] = make_float2(bu, bv);
  }
}

// ---- DIA CG ------------------------------------------------------------------
struct DiaArgs {
  const float *pl;  // 2G + 1 planes, plane stride ps
  size_t ps;
  int D, H, W, P;
  int block;  // 1: 2x2 block Jacobi ('backslash'), 0: scalar Jacobi ('pcg')
  const float2 *b;
  float2 *x, *r, *p, *z, *q;
  double *part;  // [2 ping-pong][3][PCG_MAX_BLOCKS] (rz, rr, bb) then [2][PCG_MAX_BLOCKS] (pq)
  PcgState *st;
  double atol;   // stop when ||r|| < atol (scipy: rtol ||b||)
  int maxiter;
};

__device__ __forceinline__ float2 dia_apply(const DiaArgs &a, const float2 *__restrict__ v, int i, int j, size_t k) {
  const int D = a.D, S = 2 * D + 1, G = S * S;
  float su = 0.f, sv = 0.f;
  for (int di = -D; di <= D; ++di) {
    const int ii = i + di;
    if (ii < 0 || ii >= a.H) continue;
    for (int dj = -D; dj <= D; ++dj) {
      const int jj = j + dj;
      if (jj < 0 || jj >= a.W) continue;
      const int e = (di + D) * S + (dj + D);
      const float2 n = v[(size_t)ii * a.P + jj];
      su += a.pl[(size_t)e * a.ps + k] * n.x;
      sv += a.pl[(size_t)(G + e) * a.ps + k] * n.y;
    }
  }
  const float cuv = a.pl[(size_t)(2 * G) * a.ps + k];
  const float2 c = v[k];
  return make_float2(su + cuv * c.y, sv + cuv * c.x);
}

__device__ __forceinline__ float2 dia_minv(const DiaArgs &a, size_t k, float2 r) {
  const int D = a.D, S = 2 * D + 1, G = S * S, e0 = D * S + D;
  const float d0 = a.pl[(size_t)e0 * a.ps + k], d1 = a.pl[(size_t)(G + e0) * a.ps + k];
  if (a.block) return precond<true>(d0, a.pl[(size_t)(2 * G) * a.ps + k], d1, r);
  return precond<false>(d0, 0.f, d1, r);
}

#define DIA_A(pp, v, it) ((pp) + ((size_t)((it) & 1) * 3 + (v)) * PCG_MAX_BLOCKS)
#define DIA_B(pp, it) ((pp) + 6 * PCG_MAX_BLOCKS + (size_t)((it) & 1) * PCG_MAX_BLOCKS)

// x = 0, r = b, z = M^-1 r; partials (r.z, r.r, b.b) into A[0]
__global__ __launch_bounds__(OF_BX *OF_BY) void k_dia_init(DiaArgs a) {
  __shared__ double lds[64];
  double acc[3] = {0.0, 0.0, 0.0};
  OF_FOR_PIXELS(a.H, a.W) {
    if (j >= a.W) continue;
    const size_t k = (size_t)i * a.P + j;
    const float2 b = a.b[k], z = dia_minv(a, k, b);
    a.x[k] = make_float2(0.f, 0.f);
    a.r[k] = b;
    a.z[k] = z;
    a.p[k] = make_float2(0.f, 0.f);
    acc[0] += (double)b.x * z.x + (double)b.y * z.y;
    acc[1] += (double)b.x * b.x + (double)b.y * b.y;
  }
  acc[2] = acc[1];
  write_partials<3>(acc, DIA_A(a.part, 0, 0), lds);
}

// iteration it, first half (scipy cg): stop test on ||r||; beta; p = z + beta
// p; q = A p; partial p.q
__global__ __launch_bounds__(OF_BX *OF_BY) void k_dia_dir(DiaArgs a, int it, int nb) {
  __shared__ double lds[64];
  __shared__ int s_exit;
  if (a.st->done) return;
  double s[3];
  prologue_sum<3>(s, DIA_A(a.part, 0, it), nb, lds);
  const double rz = s[0], rr = s[1];
  const int tid = threadIdx.x + threadIdx.y * blockDim.x;
  const bool lead = blockIdx.x == 0 && blockIdx.y == 0;
  if (tid == 0) {
    int ex = 0;
    if (sqrt(rr) < a.atol || rr == 0.0) ex = 1;
    else if (it >= a.maxiter) ex = 2;
    else if (!(rz > 0.0) && it > 0) ex = 1;  // fp32 noise floor (see cg_prologue)
    s_exit = ex;
    if (lead) {
      a.st->rr = rr;
      a.st->iter = it;
      a.st->rho[it & 1] = rz;
      if (ex) a.st->done = ex;
    }
  }
  __syncthreads();
  if (s_exit) return;
  const float beta = it == 0 ? 0.f : (float)(rz / a.st->rho[(it - 1) & 1]);
  OF_FOR_PIXELS(a.H, a.W) {
    if (j >= a.W) continue;
    const size_t k = (size_t)i * a.P + j;
    const float2 z = a.z[k], po = a.p[k];
    a.p[k] = make_float2(z.x + beta * po.x, z.y + beta * po.y);
  }
  // q = A p reads the new p of the neighbours (a grid-wide dependency): the
  // next launch, k_dia_q
}

__global__ __launch_bounds__(OF_BX *OF_BY) void k_dia_q(DiaArgs a, int it) {
  __shared__ double lds[64];
  if (a.st->done) return;
  double acc[1] = {0.0};
  OF_FOR_PIXELS(a.H, a.W) {
    if (j >= a.W) continue;
    const size_t k = (size_t)i * a.P + j;
    const float2 q = dia_apply(a, a.p, i, j, k), p = a.p[k];
    a.q[k] = q;
    acc[0] += (double)p.x * q.x + (double)p.y * q.y;
  }
  write_partials<1>(acc, DIA_B(a.part, it), lds);
}

// iteration it, second half: alpha = rz / p.q; x += alpha p; r -= alpha q;
// z = M^-1 r; partials (r.z, r.r) of iteration it + 1
__global__ __launch_bounds__(OF_BX *OF_BY) void k_dia_upd(DiaArgs a, int it, int nb) {
  __shared__ double lds[64];
  if (a.st->done) return;
  double s[1];
  prologue_sum<1>(s, DIA_B(a.part, it), nb, lds);
  const double pq = s[0], rz = a.st->rho[it & 1];
  if (!(pq > 0.0)) {  // fp32 underflow of p.Ap (see cg_prologue)
    if (threadIdx.x == 0 && threadIdx.y == 0 && blockIdx.x == 0 && blockIdx.y == 0) a.st->done = 1;
    return;
  }
  const float alpha = (float)(rz / pq);
  double acc[3] = {0.0, 0.0, 0.0};
  OF_FOR_PIXELS(a.H, a.W) {
    if (j >= a.W) continue;
    const size_t k = (size_t)i * a.P + j;
    const float2 p = a.p[k], q = a.q[k], x = a.x[k], r0 = a.r[k];
    a.x[k] = make_float2(x.x + alpha * p.x, x.y + alpha * p.y);
    const float2 r = make_float2(r0.x - alpha * q.x, r0.y - alpha * q.y);
    a.r[k] = r;
    const float2 z = dia_minv(a, k, r);
    a.z[k] = z;
    acc[0] += (double)r.x * z.x + (double)r.y * z.y;
    acc[1] += (double)r.x * r.x + (double)r.y * r.y;
  }
  write_partials<3>(acc, DIA_A(a.part, 0, it + 1), lds);
}

// fp64 true residual t = b - A x (stored as fp32 in t), partials ||t||^2
__global__ __launch_bounds__(OF_BX *OF_BY) void k_dia_resid(DiaArgs a, float2 *t) {
  __shared__ double lds[64];
  const int D = a.D, S = 2 * D + 1, G = S * S;
  double acc[1] = {0.0};
  OF_FOR_PIXELS(a.H, a.W) {
    if (j >= a.W) continue;
    const size_t k = (size_t)i * a.P + j;
    double su = a.b[k].x, sv = a.b[k].y;
    for (int di = -D; di <= D; ++di) {
      const int ii = i + di;
      if (ii < 0 || ii >= a.H) continue;
      for (int dj = -D; dj <= D; ++dj) {
        const int jj = j + dj;
        if (jj < 0 || jj >= a.W) continue;
        const int e = (di + D) * S + (dj + D);
        const float2 n = a.x[(size_t)ii * a.P + jj];
        su -= (double)a.pl[(size_t)e * a.ps + k] * n.x;
        sv -= (double)a.pl[(size_t)(G + e) * a.ps + k] * n.y;
      }
    }
    const double cuv = a.pl[(size_t)(2 * G) * a.ps + k];
    su -= cuv * a.x[k].y;
    sv -= cuv * a.x[k].x;
    t[k] = make_float2((float)su, (float)sv);
    acc[0] += su * su + sv * sv;
  }
  write_partials<1>(acc, a.part + 8 * PCG_MAX_BLOCKS, lds);
}

__global__ void k_dia_sum(const double *part, int nb, double *out) {
  __shared__ double lds[64];
  double s[1];
  prologue_sum<1>(s, part, nb, lds);
  if (threadIdx.x == 0 && threadIdx.y == 0) *out = s[0];
}

// x += e (iterative refinement of the 'backslash' surrogate)
__global__ __launch_bounds__(OF_BX *OF_BY) void k_dia_acc(float2 *x, const float2 *__restrict__ e, int H, int W,
                                                           int P) {
  OF_FOR_PIXELS(H, W) {
    if (j >= W) continue;
    const size_t k = (size_t)i * P + j;
    x[k] = make_float2(x[k].x + e[k].x, x[k].y + e[k].y);
  }
}

// ---- DIA lexicographic SOR (base.py:138-172) ---------------------------------
// Rows in the reference's vector order: all u rows (k = j H + i, column-major),
// then all v rows.  One workgroup walks a column wavefront: thread t owns
// column cb*nt + t and at step s updates row i = s - L t (L = D + 1), so every
// neighbour a stencil row reads is already updated when it precedes the row in
// the lexicographic order and not yet updated when it follows it.  One
// barrier per step; the sweep's |x - x_old|^2 and |x|^2 in fp64, reduced in a
// fixed order.  x must be zero on entry.
__global__ __launch_bounds__(1024) void k_dia_sor(DiaArgs a, float omega, int maxit, double tol) {
  __shared__ double red[2][16];
  const int t = threadIdx.x, nt = blockDim.x;
  const int D = a.D, S = 2 * D + 1, G = S * S, e0 = D * S + D, L = D + 1;
  int sweep = 0;
  bool conv = false;  // the stopping test passed (also on the last allowed sweep)
  for (; sweep < maxit; ++sweep) {
    double dn = 0.0, xn = 0.0;
    for (int comp = 0; comp < 2; ++comp) {
      const float *cpl = a.pl + (size_t)(comp ? G : 0) * a.ps;
      const float *cuv = a.pl + (size_t)(2 * G) * a.ps;
      for (int cb = 0; cb * nt < a.W; ++cb) {
        const int ncol = min(nt, a.W - cb * nt), j = cb * nt + t;
        const int nsteps = a.H + L * (ncol - 1);
        for (int s = 0; s < nsteps; ++s) {
          const int i = s - L * t;
          if (t < ncol && i >= 0 && i < a.H) {
            const size_t k = (size_t)i * a.P + j;
            const float dg = cpl[(size_t)e0 * a.ps + k];
            float *xc = reinterpret_cast<float *>(a.x) + comp;
            const float old = xc[2 * k];
            float nw = old;
            if (fabsf(dg) >= 1e-15f) {
              float sig = 0.f;
              for (int di = -D; di <= D; ++di) {
                const int ii = i + di;
                if (ii < 0 || ii >= a.H) continue;
                for (int dj = -D; dj <= D; ++dj) {
                  const int jj = j + dj;
                  if (jj < 0 || jj >= a.W || (di == 0 && dj == 0)) continue;
                  sig += cpl[(size_t)((di + D) * S + (dj + D)) * a.ps + k] * xc[2 * ((size_t)ii * a.P + jj)];
                }
              }
              sig += cuv[k] * reinterpret_cast<const float *>(a.x)[2 * k + (1 - comp)];
              const float bk = reinterpret_cast<const float *>(a.b)[2 * k + comp];
              nw = (1.0f - omega) * old + omega * (bk - sig) / dg;
              xc[2 * k] = nw;
            }
            dn += (double)(nw - old) * (nw - old);
            xn += (double)nw * nw;
          }
          __syncthreads();
        }
      }
    }
    // fixed-order block reduction of (dn, xn)
    dn = wave_sum(dn);
    xn = wave_sum(xn);
    if ((t & 63) == 0) {
      red[0][t >> 6] = dn;
      red[1][t >> 6] = xn;
    }
    __syncthreads();
    double sd = 0.0, sx = 0.0;
    for (int w = 0; w < nt / 64; ++w) {
      sd += red[0][w];
      sx += red[1][w];
    }
    __syncthreads();
    if (sqrt(sd) < tol * sqrt(sx)) {
      ++sweep;
      conv = true;
      break;
    }
  }
  if (t == 0) {
    a.st->iter = sweep;
    a.st->done = conv ? 1 : 2;
  }
}
