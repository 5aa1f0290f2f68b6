// kernels.h — kernel-argument PODs shared by the kernel files and the driver.
#pragma once
#include "common.h"

#define OF_BSPL_K 16

struct Taps {  // small correlation kernel (<= 5x5)
  float w[25];
  int kh, kw;
};

struct BsplTaps {
  float h[OF_BSPL_K + 1];
};

// Flow-operator parameters (classic_nl.py:279-378 / ba.py:208-302 /
// hs.py:144-203 / alt_ba.py:236-242) flattened for the assembly kernel.
struct OpArgs {
  PenF qd, qsu[2], qsv[2];  // quadratic relaxation
  PenF rd, rsu[2], rsv[2];  // robust
  PenF rc;                  // AltBA coupling
  float aq_s, ar_s;         // spatial blend: alpha*lambda_q, (1-alpha)*lambda
  float aq_d, ar_d;         // data blend: alpha, 1-alpha
  int use_q, use_r;
  float lambda2;            // AltBA coupling weight (0 = off)
  // k_flow_operator_f64: the blend factors and lambda2 unrounded
  int f64;
  double aq_s_d, ar_s_d, aq_d_d, ar_d_d, lambda2_d;
};

// Per-level derivative planes: for channel c (pointers already offset)
struct DerivArgs {
  const float *I1, *I2;          // images (nc planes each, plane stride ps)
  const float *I1x, *I1y;        // frame-1 derivative grids
  const float *A, *B, *Cc;       // interp-specific planes of frame 2:
                                 //  bi-cubic : DX, DY, DXY
                                 //  cubic    : B-spline coefs of I2x, I2y, and I2 (in Cc)
                                 //  bi-linear: I2x, I2y, -
  int nc;
  float blend;
};

// PCG scalar state (device-resident; mirrored to pinned host memory)
// CG progress mirrored to mapped, coherent host memory by the lead block of
// every launch: the host feeds launches a few ahead of `k` and stops as soon
// as `done` is set (no event round trip, few no-op launches)
struct CgFlag {
  int k;      // last launch whose prologue ran
  int done;   // PcgState::done once decided
  int iter;
  int upd;    // the 'backslash' solve's residual replacement (k_cg_update) has run
};

struct PcgState {
  double rho[2];    // r.z of iterate k at rho[k & 1]
  double rr;        // r.r
  double atol;      // rtol * ||b||
  double bnorm;
  float alpha, beta;
  int iter;
  int done;         // 0 running, 1 converged, 2 maxiter, 3 zero rhs
  int maxiter;
  // 'backslash' residual replacement: index of the CG launch that follows
  // the k_cg_update that acted (0: none yet).  That launch starts x_lo from
  // 0 and takes r.r from the update; x = x_hi + x_lo from then on.
  int upd_k;
  // launch whose prologue first saw ||r|| < upd_rel ||b|| (0: not yet): the
  // replacement offered after it acts
  int upd_due;
  int pad_;
  double xnorm2, dnorm2;  // SOR
};
