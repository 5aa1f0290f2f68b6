/*
 * optflow.h — C ABI of the MI355X-native variational optical-flow solver.
 *
 * One shared library (liboptflow.so, HIP for gfx950) runs the reference's
 * coarse-to-fine IRLS inner loop on the GPU.  The Python package
 * `optical_flow` (same API as jordanshivers/optical-flow-python) binds these
 * symbols with ctypes; any other host language binds the same symbols (see
 * INTEGRATION.md).  No torch / CUDA types appear here: plain pointers, sizes
 * and POD structs only.
 *
 * Conventions
 *   - Host buffers are caller-owned, C-contiguous float32.  "planar" means
 *     channel-major: plane c of an HxW image starts at c*H*W.  Flow fields
 *     (uv) are planar too: u plane then v plane.
 *   - Every function returns 0 on success and a negative OF_E* code on error;
 *     of_last_error() returns a message for the calling thread's context.
 *   - A context binds one HIP device and one stream; one context per host
 *     thread.  Calls are synchronous with respect to host buffers.
 *   - Non-convergence of an iterative solve is reported (of_stats), never an
 *     error — matching the reference, which ignores cg's `info`
 *     (optical_flow/methods/base.py:134-136).
 */
#ifndef OPTFLOW_H
#define OPTFLOW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OF_ABI_VERSION 3

/* status codes */
#define OF_OK 0
#define OF_EINVAL (-1)   /* bad argument (ValueError in the Python mirror) */
#define OF_EHIP (-2)     /* HIP runtime error */
#define OF_ENOMEM (-3)
#define OF_ENOTSUP (-4)  /* valid in the reference but not supported here */
#define OF_ERCCL (-5)

/* method kinds: optical_flow/methods/{hs,ba,classic_nl,alt_ba}.py */
enum of_method { OF_METHOD_HS = 0, OF_METHOD_BA = 1, OF_METHOD_CLASSIC_NL = 2, OF_METHOD_ALT_BA = 3 };

/* interpolation_method (optical_flow/utils/derivatives.py:148-294) */
enum of_interp { OF_INTERP_CUBIC = 0 /* 'cubic' = cubic B-spline */,
                 OF_INTERP_BICUBIC = 1 /* 'bi-cubic' = Hermite */,
                 OF_INTERP_BILINEAR = 2 /* 'bi-linear' */ };

/* solver (optical_flow/methods/base.py:87-114) */
enum of_solver { OF_SOLVER_BACKSLASH = 0, OF_SOLVER_PCG = 1, OF_SOLVER_SOR = 2 };

/* robust penalties (optical_flow/robust/penalties.py); OF_PEN_CONST is an
 * internal kind: rho'(x)/x == p0 everywhere (Horn-Schunck's 1/sigma^2). */
enum of_penalty_kind {
  OF_PEN_QUADRATIC = 0, OF_PEN_LORENTZIAN = 1, OF_PEN_CHARBONNIER = 2,
  OF_PEN_GEN_CHARBONNIER = 3, OF_PEN_GEMAN_MCCLURE = 4, OF_PEN_HUBER = 5,
  OF_PEN_TUKEY = 6, OF_PEN_GAUSSIAN = 7, OF_PEN_TDIST = 8, OF_PEN_TDIST_UNNORM = 9,
  OF_PEN_CONST = 100
};

typedef struct of_penalty {
  int32_t kind;
  int32_t pad_;
  double p0;   /* sigma, or r for t-dist */
  double p1;   /* a for generalized charbonnier, s for t-dist */
} of_penalty;

/*
 * A general spatial_filters list (classic_nl.py:301-322, ba.py:228-246,
 * alt_ba.py:298-316): filter i is fh[i] x fw[i] taps (row-major, at most
 * 5 x 5), applied as the reference's make_convn_mat(F, sz, 'valid',
 * 'sameswap') (utils/sparse_ops.py:59-109) with its own penalties.  general
 * = 0 means the default pair [[1, -1]], [[1], [-1]] with rho_spatial_* /
 * qua_spatial_* of of_params (the matrix-free 5-point hot path).
 */
#define OF_MAX_FILTERS 8
#define OF_MAX_FDIM 5
typedef struct of_filter_set {
  int32_t general;
  int32_t n;
  int32_t fh[OF_MAX_FILTERS], fw[OF_MAX_FILTERS];
  double taps[OF_MAX_FILTERS][OF_MAX_FDIM * OF_MAX_FDIM];
  of_penalty rho_u[OF_MAX_FILTERS], rho_v[OF_MAX_FILTERS];
  of_penalty qua_u[OF_MAX_FILTERS], qua_v[OF_MAX_FILTERS];
} of_filter_set;

/*
 * POD mirror of the method object's attribute bag
 * (optical_flow/methods/base.py:21-63, hs.py:23-47, ba.py:26-55,
 *  classic_nl.py:32-87, alt_ba.py:31-79).  The Python mirror fills it.
 */
typedef struct of_params {
  int32_t method;            /* enum of_method */
  int32_t solver;            /* enum of_solver */
  int32_t interp;            /* enum of_interp */
  int32_t texture;           /* ROF structure-texture pre-pass */
  int32_t fc;                /* high-pass pre-filter */
  int32_t auto_level;        /* BA/NL: pyramid_levels from image size */
  int32_t pyramid_levels;
  int32_t gnc_iters;
  int32_t gnc_pyramid_levels;
  int32_t max_iters;         /* IRLS warping iterations (BA, NL, AltBA) */
  int32_t max_warping_iters; /* HS */
  int32_t max_linear;
  int32_t pcg_maxiter;
  int32_t sor_max_iters;
  int32_t limit_update;
  int32_t median_filter_size;   /* 0 = None, else odd square size (5) */
  int32_t mf_iter;              /* HS */
  int32_t use_wmf;              /* Classic+NL non-local weighted median */
  int32_t area_hsz;
  int32_t itersLO;              /* AltBA */
  int32_t exact_maxiter;        /* 'backslash' surrogate: max PCG iterations */
  int32_t display;
  int32_t guide_mode;           /* estimate_flow builds a colour guide (color_images is not None) */
  int32_t pad_;
  double lambda_;
  double lambda_q;
  double alpha;                 /* initial GNC alpha */
  double pyramid_spacing;
  double gnc_pyramid_spacing;
  double pcg_rtol;
  double exact_rtol;            /* 'backslash' surrogate tolerance */
  double sor_omega;
  double sor_tol;
  double blend;
  double alp;
  double sigma_i;
  double sigmaD2, sigmaS2;      /* HS */
  double lambda2, lambda3;      /* AltBA */
  double deriv_filter[5];
  of_penalty rho_data, rho_spatial_u[2], rho_spatial_v[2];
  of_penalty qua_data, qua_spatial_u[2], qua_spatial_v[2];  /* quadratic relaxation */
  of_penalty rho_couple;        /* AltBA */
  of_filter_set filters;        /* ABI 3: general spatial_filters */
} of_params;

/* per-call statistics (may be NULL) */
#define OF_MAX_LEVELS 32
typedef struct of_stats {
  int32_t n_levels;                  /* levels processed (all GNC stages) */
  int32_t level_h[OF_MAX_LEVELS];
  int32_t level_w[OF_MAX_LEVELS];
  int32_t level_stage[OF_MAX_LEVELS];
  double level_ms[OF_MAX_LEVELS];    /* wall time of one compute_flow_base */
  int32_t solves;
  int32_t solver_iters_total;
  int32_t solver_iters_max;
  int32_t solves_not_converged;
  double total_ms;
  double preprocess_ms;
} of_stats;

typedef struct of_ctx of_ctx;

/* ---- context ---- */
int of_abi_version(void);
int of_device_count(int *count);
int of_ctx_create(int device, of_ctx **out);
int of_ctx_destroy(of_ctx *ctx);
const char *of_last_error(of_ctx *ctx);
int of_synchronize(of_ctx *ctx);
/* per-kernel HIP-event timing on the ctx stream: 0 = off, 1 = keyed by kernel
 * name, 2 = keyed by "name@pixels" (one entry per kernel and level size);
 * 3 = as 2, and every launch's start / end is also kept on a common time
 * axis across the batch lanes (of_kernel_timeline); see of_kernel_times */
int of_set_profiling(of_ctx *ctx, int enable);
/* solver options of a context (inherited by its batch lanes):
 *   OF_OPT_SOR_PIPELINE  2 (default): 'sor' runs its sweeps pipelined in one
 *                        persistent launch (k_sor_pipe), and a level of <= 64
 *                        rows whose LDS ring holds >= 8 sweeps in one
 *                        workgroup (k_sor_wg); 1: k_sor_pipe only; 0: one
 *                        launch per sweep
 *                        (k_sor_lex).  All give the same iterate and sweep
 *                        count bitwise. */
#define OF_OPT_SOR_PIPELINE 1
/*   OF_OPT_FUSED_WARP    1 (default): each warping iteration's partial_deriv
 *                        and flow_operator run as one kernel (no It / Ix /
 *                        Iy planes; 1 or 3 channels, one linearisation per
 *                        warp); 0: two kernels.  The same system bitwise
 *                        (no fma contraction in either form's warp, weight
 *                        and assembly arithmetic; tests/test_gpu_stages.py). */
#define OF_OPT_FUSED_WARP 3
int of_set_option(of_ctx *ctx, int option, int value);
/* read an option, or a read-only counter of the context and its batch lanes:
 *   OF_OPT_SOR_FALLBACKS  pipelined SOR solves whose sweep hand-off timed out
 *                         and were redone by the per-sweep kernel (the same
 *                         result; a sign of an oversubscribed GPU) */
#define OF_OPT_SOR_FALLBACKS 2
/*   OF_OPT_DEVICE_BYTES   device bytes the context and its batch lanes hold in
 *                         grow-only buffers (arena, SOR sweep ring, gather
 *                         buffer): flat across repeated pairs of one size */
#define OF_OPT_DEVICE_BYTES 4
/*   OF_OPT_RCCL_NRANKS    ranks of the context's RCCL communicator as RCCL
 *                         reports them (ncclCommCount; 0 before of_rccl_init) */
#define OF_OPT_RCCL_NRANKS 5
int of_get_option(of_ctx *ctx, int option, int64_t *value);
/* progress of compute_flow / compute_flow_base: the reference's `display`
 * prints and its per-GNC-stage report (classic_nl.py:141-196, 255-256;
 * ba.py:101-133, 189-190; hs.py:80-81, 123-124; alt_ba.py:128-183, 249-250).
 * The callback runs on the calling thread, synchronously, between kernel
 * launches.  Events: a GNC stage starts; a pyramid level starts; a warping /
 * linear iteration's solve is done (with OF_PROGRESS_ITER: `norm` = the
 * reference's ||x - duv|| after the clip, or HS's ||x||, in fp64 on the
 * device -- one stream synchronisation per iteration); a GNC stage ends
 * (`elapsed_s` after a stream synchronisation; with OF_PROGRESS_FLOW `uv`
 * holds the stage's flow, planar 2 x h x w, valid during the call).  Batch
 * entries (of_pairs_*) never report.  fn = NULL turns it off. */
enum of_event { OF_EV_STAGE = 0, OF_EV_LEVEL = 1, OF_EV_ITER = 2, OF_EV_STAGE_END = 3 };
#define OF_PROGRESS_ITER 1
#define OF_PROGRESS_FLOW 2
typedef struct of_progress {
  int32_t event;           /* enum of_event */
  int32_t stage;           /* GNC stage, 0-based */
  int32_t level;           /* pyramid level index l (0 = finest; -1 for compute_flow_base) */
  int32_t h, w;            /* level size */
  int32_t iter, lin;       /* warping iteration i, linear iteration j (0-based) */
  int32_t pad_;
  double norm;             /* OF_EV_ITER */
  double elapsed_s;        /* OF_EV_STAGE_END: seconds since compute_flow started */
  const float *uv;         /* OF_EV_STAGE_END with OF_PROGRESS_FLOW, else NULL */
} of_progress;
typedef void (*of_progress_fn)(void *user, const of_progress *ev);
int of_set_progress(of_ctx *ctx, of_progress_fn fn, void *user, int flags);
/* kernel timing accumulated since enable: per kernel name total ms, launch
 * count and pixels processed (sum over launches of the level's H*W; ROF
 * counts H*W*channels); any output pointer may be NULL */
int of_kernel_times(of_ctx *ctx, int max, const char **names, double *ms, int64_t *count, double *pixels, int *n);
/* profiling mode 3: launches since enable, each with its kernel name, level
 * pixels and [start, end] in ms after the enable call (HIP events; lanes of a
 * batch share the time axis); *n = number of launches recorded */
int of_kernel_timeline(of_ctx *ctx, int max, const char **names, double *pixels, double *t0_ms, double *t1_ms,
                       int *n);

/*
 * Whole pair: estimate_flow (optical_flow/interface.py:11-71) without its
 * Python-side parameter handling.
 *   im1, im2 : H x W x C interleaved float32, C == 1 (gray) or C == 3 (RGB;
 *              converted on device with _rgb2gray / _rgb2lab semantics)
 *   init_uv  : planar 2 x H x W or NULL (zeros)
 *   out_uv   : planar 2 x H x W
 * The final GNC alpha is written back to params->alpha (Classic+NL keeps it,
 * classic_nl.py:180-184; BA restores it, ba.py:136).
 */
int of_estimate_flow(of_ctx *ctx, of_params *params, const float *im1, const float *im2,
                     int H, int W, int C, const float *init_uv, float *out_uv, of_stats *stats);

/*
 * compute_flow() on an already preprocessed pair (the method object's
 * `images`, `color_images`):
 *   images : planar (2*nc) x H x W   (frame-1 channels then frame-2 channels)
 *   guide  : planar gc x H x W Lab/gray guide for the weighted median, or NULL
 */
int of_compute_flow(of_ctx *ctx, of_params *params, const float *images, int H, int W, int nc,
                    const float *guide, int gc, const float *init_uv, float *out_uv, of_stats *stats);

/* compute_flow_base() for one pyramid level with the given alpha (one call =
 * all warping iterations of the level; hs.py:109-142, ba.py:143-206,
 * classic_nl.py:200-277).  uv_in / out_uv planar 2 x H x W. */
int of_compute_flow_base(of_ctx *ctx, of_params *params, const float *images, int H, int W, int nc,
                         const float *guide, int gc, double alpha, const float *uv_in, float *out_uv);
/* AltBAOpticalFlow.compute_flow_base(uv, uvhat) (alt_ba.py:189-274): one
 * level of the coupled IRLS (lambda2 annealed 1e-4 -> lambda2 over max_iters
 * warps, coupling weights rho_couple'(uv - uvhat)/x, Li-Osher median update
 * of uvhat, uv <- uvhat when `replacement`); uv, uvhat in and out are planar
 * 2 x H x W */
int of_alt_ba_flow_base(of_ctx *ctx, of_params *params, const float *images, int H, int W, int nc, double alpha,
                        int replacement, const float *uv, const float *uvhat, float *out_uv, float *out_uvhat);

/* ---- device-resident batch path (benchmark / multi-GPU sharding) ---- */
/* upload one RGB/gray pair into slot `slot` of the ctx (H2D, untimed) */
int of_pair_upload(of_ctx *ctx, int slot, const float *im1, const float *im2, int H, int W, int C);
/* run estimate_flow on device-resident slot; result stays on device */
int of_pair_run(of_ctx *ctx, int slot, of_params *params, of_stats *stats);
/* run estimate_flow on slots 0..nslots-1 with `lanes` concurrent pipelines
 * (1..16; each its own HIP stream, device arena and solver state, driven by
 * its own host thread; slot s runs on lane s % lanes).  params is copied per
 * slot and not written back; stats (may be NULL) receives slot 0's.  Returns
 * when every slot is done.  Results: lanes == 1 is bitwise estimate_flow;
 * lanes >= 2 are bitwise equal to each other, and equal to estimate_flow for
 * pairs below 2^20 px; at >= 2^20 px their fine CG solves run two pairs side
 * by side in a different block geometry, so they differ from estimate_flow
 * by CG rounding only (both meet the 1e-6 true residual). */
int of_pairs_run(of_ctx *ctx, int nslots, const of_params *params, int lanes, of_stats *stats);
/* host-to-host batch (the SURVEY.md §8d headline; replaces a Python loop of
 * estimate_flow(im1[k], im2[k], method) calls, interface.py:11-71): reads
 * npairs caller-owned (H, W, C) uint8 frame pairs (C = 1 or 3), writes each
 * pair's flow as planar 2 x H x W fp32 into out_uv[k].  `lanes` pairs in
 * flight as in of_pairs_run; per lane the H2D of pair j+1's bytes and the
 * D2H of pair j-1's flow overlap pair j's kernels (pinned double buffers, one
 * copy stream shared by the lanes).  The flows also stay on the device in
 * slots 0..npairs-1 (of_pair_download, of_rccl_gather_flows); frames an
 * earlier of_pair_upload left in those slots are released (re-upload before
 * of_pair_run / of_pairs_run).  Results equal of_pairs_run on the same frames
 * with the same `lanes` (bitwise; see of_pairs_run for the lanes contract). */
int of_pairs_run_host(of_ctx *ctx, int npairs, const uint8_t *const *im1, const uint8_t *const *im2, int H, int W,
                      int C, const of_params *params, int lanes, float *const *out_uv, of_stats *stats);
/*
 * Streaming host-to-host batch (the reference's per-pair loop over files,
 * flo_io.py:46-113 / metrics.py:5-53, with host I/O overlapped): a pool of
 * `lanes` pipelines (child contexts, one host thread each; lanes >= 2 share
 * the fine-solve token as of_pairs_run) takes (H, W, C) uint8 pairs from a
 * queue, so the lanes never drain between the caller's submissions.
 *   of_pairs_open   start the pool for one frame shape and parameter set
 *   of_pairs_submit queue n pairs; returns at once; the caller keeps im1[k],
 *                   im2[k] and out_uv[k] (planar 2 x H x W fp32) alive until
 *                   the pair is waited for; *first_ticket (may be NULL)
 *                   receives the first pair's ticket, the others follow
 *   of_pairs_wait   block until that pair's flow is in its out_uv
 *   of_pairs_close  finish the queued pairs, stop and free the pool
 * Flows equal of_pairs_run_host's with the same `lanes` bitwise.  While a
 * stream is open the context's compute entries (of_pairs_run,
 * of_pairs_run_host, the stage entries ...) and its settings and profiling
 * calls (of_set_option, of_set_profiling, of_set_solve_log, of_kernel_times,
 * of_kernel_timeline) return OF_EINVAL: lane 0 of the pool is the context.
 */
int of_pairs_open(of_ctx *ctx, int H, int W, int C, const of_params *params, int lanes);
int of_pairs_submit(of_ctx *ctx, int n, const uint8_t *const *im1, const uint8_t *const *im2, float *const *out_uv,
                    int64_t *first_ticket);
int of_pairs_wait(of_ctx *ctx, int64_t ticket);
int of_pairs_close(of_ctx *ctx);
/* the same pool over device-resident pairs: queue the pairs of n slots of
 * this context (of_pair_upload; frame size = the stream's); each flow stays
 * in its slot (of_pair_download, of_rccl_gather_slots).  A slot queued and
 * not yet finished is refused by of_pairs_submit_slots, of_pair_upload and
 * of_pair_download (OF_EINVAL) until its ticket is done.  Tickets
 * share the host submissions' sequence; flows equal of_pairs_run's with the
 * same `lanes` bitwise (the bench's HBM-resident rate: consecutive batches
 * queued back to back, so the lanes never drain between them). */
int of_pairs_submit_slots(of_ctx *ctx, int n, const int *slots, int64_t *first_ticket);
/* D2H of a slot's flow (planar 2 x H x W) */
int of_pair_download(of_ctx *ctx, int slot, float *out_uv);

/* ---- RCCL gather of device-resident results (one process per GPU) ---- */
int of_rccl_unique_id(char *out128);
int of_rccl_init(of_ctx *ctx, const char *id128, int nranks, int rank);
/* gather `nslots` flows (slots 0..nslots-1 of every rank) to rank 0; rank 0's
 * out_uv receives nranks*nslots planar flows (may be NULL on other ranks) */
int of_rccl_gather_flows(of_ctx *ctx, int nslots, float *out_uv_rank0);
/* the same for slots first..first+nslots-1 (rank r's slot first+s lands at
 * flow r*nslots + s) */
int of_rccl_gather_slots(of_ctx *ctx, int first, int nslots, float *out_uv_rank0);
int of_rccl_finalize(of_ctx *ctx);

/* ---- solver diagnostics ---- */
/* Launch geometry of the iterative solver kernels for an H x W level (no
 * device needed): CG ('backslash' k_cgs, 'pcg' k_cg) strips x bands, or the
 * SOR kernel's 64-row strips (grid_x = 2 * strips).  OF_ENOTSUP when the
 * level is too large for the kernel (too wide for the partial-sum slots /
 * too tall for the SOR hand-off words). */
typedef struct of_cg_geometry {
  int32_t grid_x, grid_y;  /* launch grid (blocks) */
  int32_t rows;            /* rows per band */
  int32_t bands;
  int32_t blocks;          /* grid_x * grid_y */
  int32_t strip_cols;      /* output columns per strip */
} of_cg_geometry;
int of_solver_geometry(int H, int W, int solver, of_cg_geometry *out);

/* Solve log: with it on, every linear solve (_solve_linear_system,
 * base.py:87-172) is followed by an fp64 evaluation of its TRUE relative
 * residual ||b - A x|| / ||b|| from the fp32 operator; records keep the
 * solver's own estimate beside it (CG: the recurrence residual; SOR: the
 * last sweep's ||dx|| / ||x||).  true_rel is the residual of the solver's
 * iterate ('backslash': x_hi + x_lo summed in fp64 after its residual
 * replacement, the quantity its stopping test approximates), true_rel_out
 * that of the fp32 x it returns (the same for 'pcg' and 'sor'; for
 * 'backslash' it includes the rounding of the solution to fp32, whose
 * residual alone is ~2e-6 on Classic+NL robust stages, tools/fp32_floor.py).
 * Enabling clears the log; at most 4096 records per context.  Diagnostic
 * only: adds small launches per solve. */
typedef struct of_solve_record {
  int32_t h, w;
  int32_t solver;   /* enum of_solver */
  int32_t iters;    /* CG iterations / SOR sweeps */
  int32_t done;     /* 1 converged, 2 iteration limit, 3 zero rhs */
  int32_t pad_;
  double true_rel;      /* ||b - A x|| / ||b||, fp64, of the solver's iterate */
  double est_rel;
  double true_rel_out;  /* ... of the returned fp32 x */
} of_solve_record;
int of_set_solve_log(of_ctx *ctx, int enable);
int of_solve_log(of_ctx *ctx, int max, of_solve_record *out, int *n);

/* ---- stage entries (one per hot-path row of SURVEY.md §8a; parity tests) ---- */
/* _rgb2gray + _rgb2lab + per-channel scale_image (interface.py:49-64,74-141) */
int of_preprocess(of_ctx *ctx, const float *rgb1, const float *rgb2, int H, int W,
                  float *gray_pair /*2xHxW*/, float *lab /*3xHxW*/);
/* structure_texture_decomposition_rof (utils/image_processing.py:52-136) */
int of_rof_texture(of_ctx *ctx, const float *im, int H, int W, int C, double theta, int iters,
                   double alp, float *out);
/* compute_image_pyramid level l+1 from level l (utils/pyramid.py:44-73) */
int of_pyramid_level(of_ctx *ctx, const float *im, int H, int W, int C, const double *kern, int ksize,
                     double ratio, float *out, int *outH, int *outW);
/* resample_flow (utils/warping.py:6-45) */
int of_resample_flow(of_ctx *ctx, const float *uv, int H, int W, int nH, int nW, float *out);
/* partial_deriv (utils/derivatives.py:148-296): images planar 2*nc */
int of_partial_deriv(of_ctx *ctx, const float *images, int H, int W, int nc, const float *uv,
                     int interp, const double *deriv_filter, double blend,
                     float *It, float *Ix, float *Iy);
/* flow_operator, matrix-free (classic_nl.py:279-378, ba.py:208-302, hs.py:144-203):
 * coef = 7 planes {wx_u, wy_u, wx_v, wy_v, a_uu, a_uv, a_vv}, rhs = planes {b_u, b_v}.
 * wx_* / wy_* are the (lambda-scaled) weights of the edge to the right / below. */
int of_flow_operator(of_ctx *ctx, const of_params *params, double alpha, const float *uv,
                     const float *duv, const float *It, const float *Ix, const float *Iy,
                     int H, int W, int nc, float *coef, float *rhs);
/* _solve_linear_system (base.py:87-172) on the matrix-free operator */
int of_solve(of_ctx *ctx, const of_params *params, const float *coef, const float *rhs, int H, int W,
             float *x, int *iters, double *rel_residual);
/* General spatial_filters (params->filters.general): the operator in
 * diagonal (DIA) form on the dense offset grid of radius D = max filter
 * dimension - 1, G = (2D + 1)^2 offsets (di, dj) in row-major order
 * (di = -D..D outer): planes = G planes of the u-u block, G of the v-v
 * block, then the u-v coupling (offset 0); (A x)_u(i, j) = sum_o
 * c_u,o(i, j) x_u(i + di, j + dj) + c_uv(i, j) x_v(i, j).  *D_out receives D
 * (the caller sizes planes as (2 G + 1) H W floats, G from its own filters). */
int of_flow_operator_dia(of_ctx *ctx, const of_params *params, double alpha, const float *uv,
                         const float *duv, const float *It, const float *Ix, const float *Iy,
                         int H, int W, int nc, int *D_out, float *planes, float *rhs);
/* _solve_linear_system (base.py:87-172) on a DIA operator of radius D (any
 * sparse A whose u-u / v-v blocks are 2-D stencils and whose u-v block is
 * diagonal; the Python mirror converts scipy matrices) */
int of_solve_dia(of_ctx *ctx, const of_params *params, int D, const float *planes, const float *rhs,
                 int H, int W, float *x, int *iters, double *rel_residual);
/* detect_occlusion (utils/occlusion.py:6-56) */
int of_detect_occlusion(of_ctx *ctx, const float *uv, const float *images, int H, int W, int nc,
                        float *occ);
/* denoise_color_weighted_medfilt2 (utils/weighted_median.py:24-112) */
int of_weighted_median(of_ctx *ctx, const float *uv, const float *guide, int gc, const float *occ,
                       int H, int W, int area_hsz, double sigma_i, float *out);
/* flow_to_color (viz/flow_color.py:77-107): Middlebury colour coding of an
 * interleaved (H, W, 2) flow of dtype 0 = float32 or 1 = float64 into an
 * (H, W, 3) uint8 image; |u| or |v| > 1e9 is unknown (black).  has_max = 0
 * normalises by the largest known radius, else by max(max_flow, 1e-8).  The
 * arithmetic keeps numpy's dtype rules (the flow's dtype up to the wheel
 * position, float64 for the colour blend) */
int of_flow_to_color(of_ctx *ctx, const void *flow, int dtype, int H, int W, int has_max, double max_flow,
                     uint8_t *out_rgb);
/* scipy.ndimage.median_filter(size, mode='reflect') on each of `planes` planes */
int of_median_filter(of_ctx *ctx, const float *in, int H, int W, int planes, int size, float *out);

#ifdef __cplusplus
}
#endif
#endif /* OPTFLOW_H */
