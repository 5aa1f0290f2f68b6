// driver.hip — liboptflow.so: C ABI (include/optflow.h) + the on-device
// coarse-to-fine GNC x IRLS schedule.  Unity build: the kernel files are
// included here so every kernel and its host launch live in one TU.
//
// The host never touches image data between kernels: one of_estimate_flow()
// call uploads a pair, runs preprocessing, pyramids, every warping
// iteration (warp, assembly, solve, update, occlusion, weighted median) on
// one HIP stream, and downloads the flow.  The only host<->device syncs
// inside a pair are the iterative solvers' convergence checks (one pinned
// 80-byte read per chunk of iterations, double-buffered so the GPU always
// has the next chunk queued) and Horn-Schunck's ||x|| < 1e-3 early exit.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <immintrin.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kernels_img.hip"
#include "kernels_flow.hip"
#include "kernels_solve.hip"
#include "kernels_gen.hip"

namespace {

struct OfError {
  int code;
  std::string msg;
};

#define HIPCHK(x)                                                                                    \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) throw OfError{OF_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)}; \
  } while (0)
#define REQUIRE(cond, code, msg) \
  do {                           \
    if (!(cond)) throw OfError{code, msg}; \
  } while (0)

// grow-only device arena: chunks are kept across calls, offsets reset per call
// the lanes' token for fine CG solves (BigPhase below): OF_TOKEN_SLOTS
// solves may hold it at once
#ifndef OF_TOKEN_SLOTS
#define OF_TOKEN_SLOTS 2
#endif
struct Token {
  std::mutex m;
  std::condition_variable cv;
  int free = OF_TOKEN_SLOTS;
  void lock() {
    std::unique_lock<std::mutex> l(m);
    cv.wait(l, [&] { return free > 0; });
    --free;
  }
  void unlock() {
    {
      std::lock_guard<std::mutex> l(m);
      ++free;
    }
    cv.notify_one();
  }
};

struct Arena {
  struct Chunk {
    char *p;
    size_t cap, off;
  };
  std::vector<Chunk> chunks;
  void reset() {
    for (auto &c : chunks) c.off = 0;
  }
  void *alloc(size_t bytes) {
    bytes = (bytes + 255) & ~(size_t)255;
    for (auto &c : chunks)
      if (c.cap - c.off >= bytes) {
        void *r = c.p + c.off;
        c.off += bytes;
        return r;
      }
    size_t cap = bytes > ((size_t)64 << 20) ? bytes : ((size_t)64 << 20);
    char *p = nullptr;
    HIPCHK(hipMalloc(&p, cap));
    chunks.push_back({p, cap, bytes});
    return p;
  }
  void release() {
    for (auto &c : chunks) hipFree(c.p);
    chunks.clear();
  }
  size_t reserved() const {
    size_t n = 0;
    for (const auto &c : chunks) n += c.cap;
    return n;
  }
};

struct Img {  // C planar pitched fp32 planes
  float *p = nullptr;
  int H = 0, W = 0, P = 0, C = 0;
  size_t ps() const { return (size_t)H * P; }
  float *plane(int c) const { return p + (size_t)c * ps(); }
};
struct F2 {  // pitched float2 field
  float2 *p = nullptr;
  int H = 0, W = 0, P = 0;
};

struct ProfRec {
  const char *name;
  hipEvent_t e0, e1;
  double px;
};
struct KTime {
  double ms = 0, px = 0;
  int64_t n = 0;
};

struct Slot {
  void *rgb1 = nullptr, *rgb2 = nullptr;  // (H, W, C) fp32, or bytes when u8
  float *uv = nullptr;                    // dense planar 2 x H x W
  int H = 0, W = 0, C = 0;
  bool u8 = false;
  size_t cap_rgb = 0, cap_uv = 0;         // bytes of one frame, floats of uv
};

// of_pairs_run_host staging of one lane: two pinned input/output buffers and
// two device frame buffers, so pair j+1's bytes go up on the copy stream and
// pair j-1's flow comes down while pair j computes.  All lanes share the
// parent context's copy stream (`copy`, owned when own_copy): lanes + 1
// streams in all.  That fits GPU_MAX_HW_QUEUES (4) for lanes <= 3; the
// default 4 lanes oversubscribe it (5 streams, so two share a hardware queue
// and that lane's kernels and the copies queue behind each other), which was
// measured as a net gain all the same: 45.3 vs 44.4 pairs/s at 3 lanes
// (profiles/r3z_ab.log).  No copy waits on a lane's kernels inside the copy
// stream (the helper threads wait on the host).
struct HostStage {
  hipStream_t copy = nullptr;
  bool own_copy = false;
  uint8_t *pin_in[2] = {nullptr, nullptr}, *d_in[2] = {nullptr, nullptr};
  float *pin_out[2] = {nullptr, nullptr};
  hipEvent_t ev_in[2] = {nullptr, nullptr}, ev_conv[2] = {nullptr, nullptr}, ev_out[2] = {nullptr, nullptr};
  size_t cap_in = 0, cap_out = 0;
};

}  // namespace

#define OF_SOLVE_RING 256
#define OF_SLOG_MAX 4096  // solve-log entries kept per context
// lanes mode: phases on levels of at least this many pixels hold the token
#define OF_BIG_PX (double)(1 << 20)
// SOR hand-off words: a ticket counter, then [2][SOR_MAXS] progress stamps
#define OF_SOR_SYNC_BYTES (256 + 2 * SOR_MAXS * sizeof(int))
// dynamic LDS of a k_sor_lex block: unused, it keeps one block per CU (the
// measured configuration of the sc1 hand-off, MI355X_MICROARCH.md)
#define OF_SOR_SHM (96 * 1024)
// k_sor_pipe: persistent grid of one wave per CU; sync words (ticket, fail,
// stop, counters, decisions, progress stamps) then per-strip partials and the
// decided sweeps' sums
// Round-4 A/B on config 2 (tools/ab/r4_sor_ab.sh, the same flow bitwise):
// publication interval / LDS per wave (waves per CU) / grid cap: 32 / 96 KB
// (1 per CU) / 256: 7.24 pairs/s; 8 / 96 KB / 256: 9.47; 8 / 32 KB / 512:
// 12.04; 16 / 32 KB / 512: 10.23; 32 / 32 KB / 512: 7.38.  Several waves per
// CU let the batch lanes' SOR grids run side by side; a short publication
// interval lets more sweeps overlap on the 1-2-strip coarse levels.
#ifndef OF_SOR_PIPE_WAVES
#define OF_SOR_PIPE_WAVES 512
#endif
// dynamic LDS of a k_sor_pipe wave (unused): bounds the waves per CU
// k_sor_wg only where its ring holds >= OF_SORW_MIN_RING sweeps: at 60x80
// (a ring of 3) it was slower than k_sor_pipe (37 vs 32 us per sweep), at
// 30x40 (ring 8) faster (11 vs 26 us; profiles/r6e)
#ifndef OF_SORW_MIN_RING
#define OF_SORW_MIN_RING 8
#endif
// k_sor_wg's sweep ring in LDS (the rest of the 160 KB holds its stamps)
#ifndef OF_SORW_RING_BYTES
#define OF_SORW_RING_BYTES (144 * 1024)
#endif
#ifndef OF_SOR_PIPE_SHM
#define OF_SOR_PIPE_SHM (32 * 1024)
#endif
#define OF_SORP_SYNC_BYTES (1024 + SOR_RING_MAX * 2 * SOR_MAXS * sizeof(int))
#define OF_SORP_BYTES (OF_SORP_SYNC_BYTES + (SOR_RING_MAX * 2 * SOR_MAXS * 2 + SOR_RING_MAX * 2) * sizeof(double))

// Streams are plain non-blocking streams, which the runtime maps onto its
// GPU_MAX_HW_QUEUES (4 on the box) hardware queues by creation order: batch
// lanes created after other streams of the same process came and went can
// share a queue with a busy lane and serialise (8 1080p pairs x 4 lanes:
// 47.0 pairs/s with a context's lanes created first, 43.1 with them created
// after a pair pool's lanes were destroyed on that context;
// tools/order_probe.py, profiles/r5_order_probe.log).  Streams created with a
// full CU mask behaved the same (the runtime pools them too).  Keep long-lived
// lanes: a context creates its of_pairs_run lanes once and keeps them.
static void create_stream(hipStream_t *s) { HIPCHK(hipStreamCreateWithFlags(s, hipStreamNonBlocking)); }

// batch lanes created together on first use (ensure_lanes): the default 4
#ifndef OF_LANES_MIN
#define OF_LANES_MIN 4
#endif
#ifndef OF_FUSED_WARP_DEFAULT
#define OF_FUSED_WARP_DEFAULT 1
#endif
struct of_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t hp = nullptr;  // high-priority stream of fine solves (OF_SOLVE_PRIO)
  hipEvent_t ev_hp[2] = {nullptr, nullptr};
  std::string err;
  Arena arena;
  PcgState *d_state = nullptr, *h_state = nullptr;  // h_state: 2 pinned slots
  hipEvent_t ev_state[2] = {nullptr, nullptr};
  // CG solves: per-solve progress flags (mapped coherent host memory) and
  // copies of the final state (pinned), a ring of OF_SOLVE_RING; a solve's
  // statistics are read at the next stream synchronisation, so a CG solve
  // does not end in one
  CgFlag *h_flag = nullptr, *d_flag = nullptr;
  PcgState *h_ring = nullptr;
  int ring_next = 0;
  struct PendingSolve {
    int slot;
    double px;
    of_stats *st;
    const char *name;
  };
  std::vector<PendingSolve> pend;
  double *d_partials = nullptr;
  unsigned *d_sor_sync = nullptr;
  char *d_sorp = nullptr;  // k_sor_pipe sync words, partials (lazily allocated)
  // k_sor_pipe's ring of sweep buffers: one per context, grown to the largest
  // level seen (every SOR solve ends in a stream synchronisation, so the
  // ring is free again when the next solve starts)
  float2 *d_sor_ring = nullptr;
  size_t sor_ring_cap = 0;  // bytes
  int sor_fallbacks = 0;    // pipelined solves rerun per sweep (hand-off timeout)
  float *d_gather = nullptr;  // rank 0's RCCL gather receive buffer (grow-only)
  hipStream_t gstream = nullptr;  // the gather's own stream (of_rccl_gather_slots)
  size_t gather_cap = 0;
  // of_set_progress: display / per-stage report callback (never on batch lanes)
  of_progress_fn prog_fn = nullptr;
  void *prog_user = nullptr;
  int prog_flags = 0;
  int prog_stage = 0, prog_level = -1;
  std::chrono::steady_clock::time_point prog_t0;
  std::vector<float> prog_uv;  // host copy of a stage's flow (OF_PROGRESS_FLOW)
  // of_set_option(OF_OPT_SOR_PIPELINE): 2 (default) = k_sor_pipe, and
  // k_sor_wg where its LDS ring holds >= OF_SORW_MIN_RING sweeps
  int opt_sor_pipe = 2;
  int opt_fused_warp = OF_FUSED_WARP_DEFAULT;  // of_set_option(OF_OPT_FUSED_WARP)
  // solve log (of_set_solve_log): fp64 true residual of every solve
  int slog = 0;
  struct SolveLog {
    int h, w, solver, slot, iters, done;
    double est;
  };
  std::vector<SolveLog> slog_rec;
  int slog_idx = -1;       // log entry of the solve being issued (-1: none)
  bool slog_iter = false;  // ... whose iterate residual the solver logged itself
  double *d_rpart = nullptr, *d_rlog = nullptr;
  uint32_t *d_mm = nullptr;  // 32 min/max pairs
  double *d_norm = nullptr, *h_norm = nullptr;
  int prof = 0;  // 0 off, 1 per kernel, 2 per kernel and level ("name@pixels")
  std::vector<hipEvent_t> ev_pool;  // profiling events
  size_t ev_used = 0;
  std::vector<hipEvent_t> tev_pool;  // level timing events, recycled per API call
  size_t tev_used = 0;
  std::vector<ProfRec> pending;
  std::map<std::string, KTime> ktimes;
  // profiling mode 3: every launch's [start, end] in ms after `epoch` (an
  // event on the parent context's stream; lanes share it)
  struct TlRec {
    const char *name;
    double px, t0, t1;
  };
  std::vector<TlRec> tl;
  hipEvent_t epoch = nullptr;
  bool own_epoch = false;
  std::map<int64_t, int> iter_hints;  // (H, W, solver) -> last iteration count
  double cur_px = 0;  // pixels processed by the launches being issued (profiling)
  std::vector<Slot> slots;
  HostStage *hs = nullptr;      // of_pairs_run_host staging (lazily created)
  struct PairPool *pool = nullptr;  // of_pairs_open streaming batch (lanes of its own)
  std::vector<of_ctx *> lanes;  // of_pairs_run pipelines: own stream, arena and solver state
  Token big_own;                // (parent) the big-phase token its lanes share
  Token *big = nullptr;         // (lane) token held through phases of >= big_px pixels
  double big_px = 0;
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
};

namespace {

hipEvent_t pool_event(of_ctx *c) {
  if (c->ev_used == c->ev_pool.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    c->ev_pool.push_back(e);
  }
  return c->ev_pool[c->ev_used++];
}

hipEvent_t timing_event(of_ctx *c) {
  if (c->tev_used == c->tev_pool.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    c->tev_pool.push_back(e);
  }
  return c->tev_pool[c->tev_used++];
}

void flush_prof(of_ctx *c) {
  if (c->pending.empty()) return;
  HIPCHK(hipStreamSynchronize(c->stream));
  for (auto &r : c->pending) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, r.e0, r.e1));
    auto &s = c->prof >= 2 ? c->ktimes[std::string(r.name) + "@" + std::to_string((long long)r.px)]
                           : c->ktimes[r.name];
    s.ms += ms;
    s.px += r.px;
    s.n += 1;
    if (c->prof == 3 && c->epoch) {
      float a = 0, b = 0;
      HIPCHK(hipEventElapsedTime(&a, c->epoch, r.e0));
      HIPCHK(hipEventElapsedTime(&b, c->epoch, r.e1));
      c->tl.push_back({r.name, r.px, a, b});
    }
  }
  c->pending.clear();
  c->ev_used = 0;
}

template <typename K, typename... A>
void launch(of_ctx *c, const char *name, K kernel, dim3 g, dim3 b, size_t shm, A... args) {
  if (g.x == 0 || g.y == 0 || g.z == 0) return;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->prof) {
    if (c->ev_used + 2 > 8192) flush_prof(c);
    e0 = pool_event(c);
    e1 = pool_event(c);
    HIPCHK(hipEventRecord(e0, c->stream));
  }
  hipLaunchKernelGGL(kernel, g, b, shm, c->stream, args...);
  HIPCHK(hipGetLastError());
  if (c->prof) {
    HIPCHK(hipEventRecord(e1, c->stream));
    c->pending.push_back({name, e0, e1, c->cur_px});
  }
}

inline dim3 gz(const Grid2 &g, int z) { return dim3(g.grid.x, g.grid.y, z); }

Img new_img(of_ctx *c, int H, int W, int C) {
  Img m;
  m.H = H;
  m.W = W;
  m.C = C;
  m.P = of_pitch(W);
  m.p = (float *)c->arena.alloc(sizeof(float) * m.ps() * (C > 0 ? C : 1));
  return m;
}
F2 new_f2(of_ctx *c, int H, int W) {
  F2 f;
  f.H = H;
  f.W = W;
  f.P = of_pitch(W);
  f.p = (float2 *)c->arena.alloc(sizeof(float2) * (size_t)H * f.P);
  return f;
}
Img view(const Img &m, int c0, int n) {
  Img v = m;
  v.p = m.plane(c0);
  v.C = n;
  return v;
}

// host planar dense (C x H x W) -> device pitched
void upload_img(of_ctx *c, const Img &m, const float *host) {
  HIPCHK(hipMemcpy2DAsync(m.p, sizeof(float) * m.P, host, sizeof(float) * m.W, sizeof(float) * m.W,
                          (size_t)m.H * m.C, hipMemcpyHostToDevice, c->stream));
}
void download_img(of_ctx *c, const Img &m, float *host) {
  HIPCHK(hipMemcpy2DAsync(host, sizeof(float) * m.W, m.p, sizeof(float) * m.P, sizeof(float) * m.W,
                          (size_t)m.H * m.C, hipMemcpyDeviceToHost, c->stream));
}
void copy_img(of_ctx *c, const Img &dst, const Img &src) {
  HIPCHK(hipMemcpyAsync(dst.p, src.p, sizeof(float) * src.ps() * src.C, hipMemcpyDeviceToDevice, c->stream));
}
// planar host/dense-device uv <-> pitched float2
void f2_from_dense(of_ctx *c, const F2 &f, const float *dense_dev) {
  Grid2 g = grid2(f.H, f.W);
  launch(c, "planar2_to_f2", k_planar2_to_f2, g.grid, g.block, 0, dense_dev, f.p, f.H, f.W, f.P,
         (size_t)f.H * f.W);
}
void f2_to_dense(of_ctx *c, const F2 &f, float *dense_dev) {
  Grid2 g = grid2(f.H, f.W);
  launch(c, "f2_to_planar2", k_f2_to_planar2, g.grid, g.block, 0, (const float2 *)f.p, dense_dev, f.H, f.W, f.P,
         (size_t)f.H * f.W);
}
F2 upload_f2(of_ctx *c, const float *host, int H, int W) {
  F2 f = new_f2(c, H, W);
  float *d = (float *)c->arena.alloc(sizeof(float) * 2 * (size_t)H * W);
  HIPCHK(hipMemcpyAsync(d, host, sizeof(float) * 2 * (size_t)H * W, hipMemcpyHostToDevice, c->stream));
  f2_from_dense(c, f, d);
  return f;
}
void download_f2(of_ctx *c, const F2 &f, float *host) {
  float *d = (float *)c->arena.alloc(sizeof(float) * 2 * (size_t)f.H * f.W);
  f2_to_dense(c, f, d);
  HIPCHK(hipMemcpyAsync(host, d, sizeof(float) * 2 * (size_t)f.H * f.W, hipMemcpyDeviceToHost, c->stream));
}
void fill_f2(of_ctx *c, const F2 &f, float v) {
  Grid2 g = grid2(f.H, f.W);
  launch(c, "fill_f2", k_fill_f2, g.grid, g.block, 0, f.p, f.H, f.W, f.P, make_float2(v, v));
}

// ---- global scale_image over all planes of an image ------------------------
void scale_img(of_ctx *c, const Img &m, float vlow, float vhigh, int mm_slot) {
  uint32_t *mm = c->d_mm + 2 * mm_slot;
  launch(c, "mm_init", k_mm_init, dim3(1), dim3(64), 0, mm, 1);
  Grid2 gm = grid2(m.H, m.W, 256), g = grid2(m.H, m.W);
  launch(c, "minmax", k_minmax, gm.grid, gm.block, 0, (const float *)m.p, m.H, m.W, m.P, m.C, m.ps(), mm);
  launch(c, "scale", k_scale, g.grid, g.block, 0, m.p, m.H, m.W, m.P, m.C, m.ps(), (const uint32_t *)mm, vlow, vhigh);
}

// ---- correlation taps -------------------------------------------------------
Taps make_taps(const double *k, int kh, int kw) {
  Taps t;
  memset(&t, 0, sizeof(t));
  t.kh = kh;
  t.kw = kw;
  for (int a = 0; a < kh * kw; ++a) t.w[a] = (float)k[a];
  return t;
}
void correlate(of_ctx *c, const Img &in, const Img &out, const Taps &t) {
  Grid2 g = grid2(in.H, in.W);
  const bool fold1 = in.H > t.kh / 2 && in.W > t.kw / 2;  // one reflection reaches every tap
  auto go = [&](auto k) {
    launch(c, "correlate", k, gz(g, in.C), g.block, 0, (const float *)in.p, out.p, in.H, in.W, in.P, in.ps(), t);
  };
  if (fold1 && t.kh == 5 && t.kw == 5) go(k_correlate_k<5, 5>);
  else if (fold1 && t.kh == 1 && t.kw == 5) go(k_correlate_k<1, 5>);
  else if (fold1 && t.kh == 5 && t.kw == 1) go(k_correlate_k<5, 1>);
  else if (fold1 && t.kh == 3 && t.kw == 3) go(k_correlate_k<3, 3>);
  else if (fold1 && t.kh == 1 && t.kw == 3) go(k_correlate_k<1, 3>);
  else if (fold1 && t.kh == 3 && t.kw == 1) go(k_correlate_k<3, 1>);
  else go(k_correlate);
}

// fspecial('gaussian') (image_processing.py:29-49)
std::vector<double> gaussian(int size, double sigma) {
  std::vector<double> k(size * size);
  double m = (size - 1) / 2.0, mx = 0, s = 0;
  for (int a = 0; a < size; ++a)
    for (int b = 0; b < size; ++b) {
      double y = a - m, x = b - m;
      k[a * size + b] = std::exp(-(x * x + y * y) / (2 * sigma * sigma));
      mx = std::max(mx, k[a * size + b]);
    }
  for (auto &v : k) {
    if (v < 2.220446049250313e-16 * mx) v = 0;
    s += v;
  }
  if (s != 0)
    for (auto &v : k) v /= s;
  return k;
}

void resize_dims(int H, int W, double ratio, int *nH, int *nW) {
  int a = (int)std::floor(H * ratio + 0.5), b = (int)std::floor(W * ratio + 0.5);
  *nH = a < 1 ? 1 : a;
  *nW = b < 1 ? 1 : b;
}

// one compute_image_pyramid step (pyramid.py:58-67)
// a separable kh x kw kernel ky (x) kx as a row pass then a column pass
// (10 taps per pixel instead of 25 for 5 x 5; same sums, another rounding order)
void correlate_sep(of_ctx *c, const Img &in, const Img &out, const Taps &tx, const Taps &ty) {
  Img tmp = new_img(c, in.H, in.W, in.C);
  correlate(c, in, tmp, tx);
  correlate(c, tmp, out, ty);
}

Img pyramid_step(of_ctx *c, const Img &in, const Taps &tx, const Taps &ty, double ratio) {
  int nH, nW;
  resize_dims(in.H, in.W, ratio, &nH, &nW);
  Img tmp = new_img(c, in.H, in.W, in.C);
  correlate_sep(c, in, tmp, tx, ty);
  Img out = new_img(c, nH, nW, in.C);
  Grid2 g = grid2(nH, nW);
  launch(c, "resize", k_resize<float>, gz(g, in.C), g.block, 0, (const float *)tmp.p, in.H, in.W, in.P, tmp.ps(),
         out.p, nH, nW, out.P, out.ps(), 1.0f);
  return out;
}

Img pyramid_step(of_ctx *c, const Img &in, const Taps &t, double ratio) {
  int nH, nW;
  resize_dims(in.H, in.W, ratio, &nH, &nW);
  Img tmp = new_img(c, in.H, in.W, in.C);
  correlate(c, in, tmp, t);
  Img out = new_img(c, nH, nW, in.C);
  Grid2 g = grid2(nH, nW);
  launch(c, "resize", k_resize<float>, gz(g, in.C), g.block, 0, (const float *)tmp.p, in.H, in.W, in.P, tmp.ps(),
         out.p, nH, nW, out.P, out.ps(), 1.0f);
  return out;
}

// _build_pyramid (base.py:174-190)
std::vector<Img> build_pyramid(of_ctx *c, const Img &img, int levels, double spacing) {
  double sig = std::sqrt(spacing) / std::sqrt(2.0);
  int ks = 2 * (int)std::nearbyint(1.5 * sig) + 1;
  // fspecial('gaussian') is the outer product of the normalised 1-D
  // Gaussian (its eps cut-off removes nothing at these sizes: the smallest
  // entry is >= 1.8 % of the largest)
  std::vector<double> g1(ks);
  double s1 = 0.0;
  for (int b = 0; b < ks; ++b) s1 += (g1[b] = std::exp(-(b - (ks - 1) / 2.0) * (b - (ks - 1) / 2.0) / (2 * sig * sig)));
  for (auto &v : g1) v /= s1;
  const Taps tx = make_taps(g1.data(), 1, ks), ty = make_taps(g1.data(), ks, 1);
  std::vector<Img> pyr{img};
  for (int l = 1; l < levels; ++l) pyr.push_back(pyramid_step(c, pyr.back(), tx, ty, 1.0 / spacing));
  return pyr;
}

// structure_texture_decomposition_rof (image_processing.py:52-136) on all planes
Img rof_texture(of_ctx *c, const Img &in, double theta, int iters, double alp) {
  c->cur_px = (double)in.H * in.W * in.C;
  Img nrm = new_img(c, in.H, in.W, in.C);
  copy_img(c, nrm, in);
  scale_img(c, nrm, -1.0f, 1.0f, 0);
  const size_t ps = nrm.ps();  // C planes of float2 p
  float2 *p0 = (float2 *)c->arena.alloc(sizeof(float2) * ps * in.C);
  float2 *p1 = (float2 *)c->arena.alloc(sizeof(float2) * ps * in.C);
  HIPCHK(hipMemsetAsync(p0, 0, sizeof(float2) * ps * in.C, c->stream));
  Grid2 g = grid2(in.H, in.W);
  const float th = (float)theta, delta = (float)(1.0 / (4.0 * theta));
  const dim3 rg((in.W + ROF_TW - 1) / ROF_TW, (in.H + ROF_TH - 1) / ROF_TH, in.C);  // 64 x 4 blocks
  for (int it = 0; it < iters; it += ROF_K) {
    launch(c, "rof_iters", k_rof_iters, rg, g.block, 0, (const float *)nrm.p, (const float2 *)p0, p1, in.H, in.W,
           nrm.P, ps, th, delta, std::min(ROF_K, iters - it));
    std::swap(p0, p1);
  }
  Img out = new_img(c, in.H, in.W, in.C);
  launch(c, "rof_final", k_rof_final, gz(g, in.C), g.block, 0, (const float *)nrm.p, (const float2 *)p0, out.p, in.H,
         in.W, nrm.P, ps, th, (float)alp);
  scale_img(c, out, 0.0f, 255.0f, 1);
  return out;
}

// ---- per-level derivative planes ---------------------------------------------
struct LevelDeriv {
  Img I1x, I1y, A, B, Cc;
  DerivArgs args;
};

LevelDeriv level_deriv(of_ctx *c, const Img &im, int nc, int interp, const double *filt, double blend) {
  LevelDeriv L;
  Img I1 = view(im, 0, nc), I2 = view(im, nc, nc);
  Taps tx = make_taps(filt, 1, 5), ty = make_taps(filt, 5, 1);
  L.I1x = new_img(c, im.H, im.W, nc);
  L.I1y = new_img(c, im.H, im.W, nc);
  correlate(c, I1, L.I1x, tx);
  correlate(c, I1, L.I1y, ty);
  L.A = new_img(c, im.H, im.W, nc);
  L.B = new_img(c, im.H, im.W, nc);
  L.Cc = new_img(c, im.H, im.W, nc);
  correlate(c, I2, L.A, tx);
  correlate(c, I2, L.B, ty);
  if (interp == OF_INTERP_BICUBIC) {
    // DXY = correlate(I2, filt^T filt) (derivatives.py:27-145), separably:
    // the row pass is A itself
    correlate(c, L.A, L.Cc, ty);
  } else if (interp == OF_INTERP_CUBIC) {
    // B-spline coefficients of I2x, I2y (in place via tmp) and of I2 (into Cc)
    BsplTaps bt;
    const double z = std::sqrt(3.0) - 2.0, c0 = -6.0 * z / (1.0 - z * z);
    for (int k = 0; k <= OF_BSPL_K; ++k) bt.h[k] = (float)(c0 * std::pow(z, (double)k));
    Img tmp = new_img(c, im.H, im.W, nc);
    Grid2 g = grid2(im.H, im.W);
    auto pf = [&](const Img &src, const Img &dst) {
      launch(c, "bspline_rows", k_bspline_rows, gz(g, nc), g.block, 0, (const float *)src.p, tmp.p, im.H, im.W, im.P,
             im.ps(), bt);
      launch(c, "bspline_cols", k_bspline_cols, gz(g, nc), g.block, 0, (const float *)tmp.p, dst.p, im.H, im.W, im.P,
             im.ps(), bt);
    };
    pf(L.A, L.A);
    pf(L.B, L.B);
    pf(I2, L.Cc);
  }
  DerivArgs &d = L.args;
  d.I1 = I1.p;
  d.I2 = I2.p;
  d.I1x = L.I1x.p;
  d.I1y = L.I1y.p;
  d.A = L.A.p;
  d.B = L.B.p;
  d.Cc = L.Cc.p;
  d.nc = nc;
  d.blend = (float)blend;
  return L;
}

void partial_deriv(of_ctx *c, const LevelDeriv &L, int interp, const F2 &uv, const Img &It, const Img &Ix,
                   const Img &Iy) {
  Grid2 g = grid2(uv.H, uv.W);
  const size_t ps = It.ps();
  if (interp == OF_INTERP_BICUBIC)
    launch(c, "partial_deriv_hermite", k_partial_deriv<1>, g.grid, g.block, 0, L.args, (const float2 *)uv.p, uv.H,
           uv.W, uv.P, ps, It.p, Ix.p, Iy.p);
  else if (interp == OF_INTERP_CUBIC)
    launch(c, "partial_deriv_bspline", k_partial_deriv<0>, g.grid, g.block, 0, L.args, (const float2 *)uv.p, uv.H,
           uv.W, uv.P, ps, It.p, Ix.p, Iy.p);
  else
    launch(c, "partial_deriv_bilinear", k_partial_deriv<2>, g.grid, g.block, 0, L.args, (const float2 *)uv.p, uv.H,
           uv.W, uv.P, ps, It.p, Ix.p, Iy.p);
}

OpArgs op_args(const of_params *P, double alpha, double lambda2) {
  OpArgs o;
  memset(&o, 0, sizeof(o));
  o.qd = to_penf(P->qua_data);
  o.rd = to_penf(P->rho_data);
  for (int k = 0; k < 2; ++k) {
    o.qsu[k] = to_penf(P->qua_spatial_u[k]);
    o.qsv[k] = to_penf(P->qua_spatial_v[k]);
    o.rsu[k] = to_penf(P->rho_spatial_u[k]);
    o.rsv[k] = to_penf(P->rho_spatial_v[k]);
  }
  o.rc = to_penf(P->rho_couple);
  // alpha == 1: quadratic system only; alpha == 0: robust only; else blend
  // (classic_nl.py:237-248, ba.py:374-385)
  o.use_q = alpha > 0.0;
  o.use_r = alpha < 1.0;
  o.aq_s = (float)((o.use_r ? alpha : 1.0) * P->lambda_q);
  o.ar_s = (float)((o.use_q ? 1.0 - alpha : 1.0) * P->lambda_);
  o.aq_d = (float)(o.use_r ? alpha : 1.0);
  o.ar_d = (float)(o.use_q ? 1.0 - alpha : 1.0);
  o.lambda2 = (float)lambda2;
  // AltBA's robust stage (lorentzian + charbonnier(1e-3) coupling) is
  // ill-conditioned (~3.6e6): its diagonal, a sum of edge weights and a data
  // term, must be rounded once, not per fp32 operation (k_flow_operator_f64)
  o.f64 = P->method == OF_METHOD_ALT_BA;
  o.aq_s_d = (o.use_r ? alpha : 1.0) * P->lambda_q;
  o.ar_s_d = (o.use_q ? 1.0 - alpha : 1.0) * P->lambda_;
  o.aq_d_d = o.use_r ? alpha : 1.0;
  o.ar_d_d = o.use_q ? 1.0 - alpha : 1.0;
  o.lambda2_d = lambda2;
  return o;
}

// the assembly kernels' penalty mode (kernels_flow.hip, PenMode): the
// quadratic stage or a robust stage whose penalties share one kind get a
// specialised kernel, anything else the run-time form
int pen_mode(const OpArgs &o) {
  auto all = [](std::initializer_list<const PenF *> ps, int kind) {
    for (const PenF *p : ps)
      if (p->kind != kind) return false;
    return true;
  };
  if (o.use_q && !o.use_r)
    return all({&o.qd, &o.qsu[0], &o.qsu[1], &o.qsv[0], &o.qsv[1]}, OF_PEN_QUADRATIC) ? OF_PM_Q : OF_PM_ANY;
  if (o.use_r && !o.use_q) {
    const int k = o.rd.kind;
    if ((k == OF_PEN_GEN_CHARBONNIER || k == OF_PEN_CHARBONNIER || k == OF_PEN_LORENTZIAN || k == OF_PEN_CONST) &&
        all({&o.rsu[0], &o.rsu[1], &o.rsv[0], &o.rsv[1]}, k))
      return OF_PM_R(k);
  }
  return OF_PM_ANY;
}
// calls f(kernel) with the instantiation of template K for mode m
#define OF_BY_PM(m, KT, ...)                                                               \
  switch (m) {                                                                            \
    case OF_PM_Q: f(KT<__VA_ARGS__ OF_PM_Q>); break;                                      \
    case OF_PM_R(OF_PEN_GEN_CHARBONNIER): f(KT<__VA_ARGS__ OF_PM_R(OF_PEN_GEN_CHARBONNIER)>); break; \
    case OF_PM_R(OF_PEN_CHARBONNIER): f(KT<__VA_ARGS__ OF_PM_R(OF_PEN_CHARBONNIER)>); break; \
    case OF_PM_R(OF_PEN_LORENTZIAN): f(KT<__VA_ARGS__ OF_PM_R(OF_PEN_LORENTZIAN)>); break; \
    case OF_PM_R(OF_PEN_CONST): f(KT<__VA_ARGS__ OF_PM_R(OF_PEN_CONST)>); break;           \
    default: f(KT<__VA_ARGS__ OF_PM_ANY>); break;                                          \
  }

void flow_operator(of_ctx *c, const OpArgs &o, const F2 &uv, const F2 *duv, const Img &It, const Img &Ix,
                   const Img &Iy, const F2 *uvhat, const Img &coef, const F2 &rhs) {
  Grid2 g = grid2(uv.H, uv.W);
  auto f = [&](auto kern) {
    launch(c, "flow_operator", kern, g.grid, g.block, 0, o, (const float2 *)uv.p,
           (const float2 *)(duv ? duv->p : nullptr), (const float *)It.p, (const float *)Ix.p, (const float *)Iy.p,
           It.C, (const float2 *)(uvhat ? uvhat->p : nullptr), uv.H, uv.W, uv.P, coef.ps(), coef.p, rhs.p);
  };
  if (o.f64) {
    f(k_flow_operator_f64);
    return;
  }
  const int m = uvhat ? OF_PM_ANY : pen_mode(o);
  OF_BY_PM(m, k_flow_operator, )
}

// partial_deriv + flow_operator fused (k_warp_operator): no It / Ix / Iy
// planes; nc = 1 or 3 image channels, the fp32 assembly, no duv / uvhat
bool can_fuse_warp_op(const of_ctx *c, const OpArgs &o, int nc) {
  return c->opt_fused_warp && !o.f64 && (nc == 1 || nc == 3);
}
void warp_operator(of_ctx *c, const LevelDeriv &L, int interp, const OpArgs &o, const F2 &uv, const Img &coef,
                   const F2 &rhs) {
  Grid2 g = grid2(uv.H, uv.W);
  const size_t ps = coef.ps();
  REQUIRE(L.I1x.ps() == ps && L.args.nc == L.I1x.C, OF_EHIP, "warp_operator: plane strides differ");
  const float2 *u = (const float2 *)uv.p;
  const char *name = interp == OF_INTERP_BICUBIC ? "warp_operator_hermite"
                     : interp == OF_INTERP_CUBIC ? "warp_operator_bspline"
                                                 : "warp_operator_bilinear";
  auto f = [&](auto kern) { launch(c, name, kern, g.grid, g.block, 0, L.args, o, u, uv.H, uv.W, uv.P, ps, coef.p, rhs.p); };
  const int m = pen_mode(o);
  const bool one = L.args.nc == 1;
  if (interp == OF_INTERP_BICUBIC) {
    if (one) { OF_BY_PM(m, k_warp_operator, 1, 1, ) } else { OF_BY_PM(m, k_warp_operator, 1, 3, ) }
  } else if (interp == OF_INTERP_CUBIC) {
    if (one) { OF_BY_PM(m, k_warp_operator, 0, 1, ) } else { OF_BY_PM(m, k_warp_operator, 0, 3, ) }
  } else {
    if (one) { OF_BY_PM(m, k_warp_operator, 2, 1, ) } else { OF_BY_PM(m, k_warp_operator, 2, 3, ) }
  }
}

// ---- iterative solve (base.py:87-172) -----------------------------------------
struct SolveResult {
  int iters;
  int done;
  double rel;
  int slot = -1;  // >= 0: CG solve whose state is still in flight (h_ring[slot])
  double px = 0;
  const char *name = nullptr;  // fused CG kernel whose active launches profiling counts
};

// grid for the 2-pixels-per-thread solver kernels, <= PCG_MAX_BLOCKS blocks
Grid2 pair_grid(int H, int W) {
  Grid2 g;
  g.block = dim3(OF_BX, OF_BY, 1);
  int gx = (W + 2 * OF_BX - 1) / (2 * OF_BX), gy = (H + OF_BY - 1) / OF_BY;
  int cap = std::max(1, PCG_MAX_BLOCKS / gx);
  g.grid = dim3(gx, std::min(gy, cap), 1);
  g.nblocks = g.grid.x * g.grid.y;
  return g;
}

// Enqueue iterations in chunks and poll the previous chunk's state (pinned,
// double-buffered) while the current one runs.  The first chunk is sized by
// `first` (the iteration count of the last solve of the same size and
// solver, when known), the second is short, later ones grow up to
// `max_chunk`: launches enqueued after convergence (cheap no-ops, but not
// free) stay few without leaving the GPU idle while the host polls.
template <typename Enq>
int run_chunked(of_ctx *c, int maxiter, int first, int max_chunk, Enq enqueue_iter) {
  int enq = 0, chunk = first, nchunks = 0;
  while (enq < maxiter) {
    const int n = std::min(chunk, maxiter - enq);
    for (int t = 0; t < n; ++t) enqueue_iter(enq + t);
    enq += n;
    const int slot = nchunks & 1;
    HIPCHK(hipMemcpyAsync(&c->h_state[slot], c->d_state, sizeof(PcgState), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipEventRecord(c->ev_state[slot], c->stream));
    ++nchunks;
    if (nchunks >= 2) {
      HIPCHK(hipEventSynchronize(c->ev_state[slot ^ 1]));
      if (c->h_state[slot ^ 1].done) break;
    }
    chunk = nchunks == 1 ? 4 : std::min(std::max(chunk + chunk / 2, 8), max_chunk);
  }
  return enq;
}

// Feed CG launches `depth` ahead of the progress the kernels report in the
// mapped host flag; stop enqueueing as soon as a prologue has declared the
// solve done.  Returns the number of launches enqueued.
template <typename Enq>
int run_fed(of_ctx *c, volatile CgFlag *f, int nmax, int depth, Enq enqueue_iter) {
  f->done = 0;
  f->iter = 0;
  f->upd = 0;
  f->k = -1;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  int enq = 0;
  while (enq < nmax) {
    if (f->done) break;
    if (enq - f->k <= depth) {
      enqueue_iter(enq++);
      continue;
    }
    // the GPU is `depth` launches behind: wait for progress (bounded: after
    // 0.5 s drain the stream; the flag must then show every launch)
    const auto t0 = std::chrono::steady_clock::now();
    while (!f->done && enq - f->k > depth) {
      _mm_pause();
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(500)) {
        HIPCHK(hipStreamSynchronize(c->stream));
        REQUIRE(f->done || f->k == enq - 1, OF_EHIP, "CG progress flag not visible to the host");
        break;
      }
    }
  }
  return enq;
}

void drain_solves(of_ctx *c);

// iteration-count hint of the last solve with this size and solver
int& iter_hint(of_ctx *c, int H, int W, int solver) {
  return c->iter_hints[((int64_t)H << 32) | ((int64_t)W << 8) | solver];
}

// profiling: launches of a solve that did work (the rest returned after the
// prologue); bench.py prices algorithmic bytes on these
void note_active(of_ctx *c, const char *name, int launches, double px) {
  if (!c->prof) return;
  const std::string key = std::string(name) + ".active";
  auto &s = c->ktimes[c->prof >= 2 ? key + "@" + std::to_string((long long)px) : key];
  s.px += launches * px;
  s.n += launches;
}

// Coefficients c_i of the degree-m polynomial preconditioner of k_cgp,
// M^-1 = sum_i c_i B^i D^-1 with B = I - X, X = D^-1 A: the Chebyshev
// residual polynomial 1 - X p(X) = T_{m+1}((b + a - 2X) / (b - a)) /
// T_{m+1}((b + a) / (b - a)), re-expanded in powers of B.
void cheb_poly(int m, double a, double b, double *cB) {
  std::vector<std::vector<double>> T(m + 2);
  T[0] = {1.0};
  T[1] = {0.0, 1.0};
  for (int i = 2; i <= m + 1; ++i) {
    T[i].assign(i + 1, 0.0);
    for (size_t j = 0; j < T[i - 1].size(); ++j) T[i][j + 1] += 2.0 * T[i - 1][j];
    for (size_t j = 0; j < T[i - 2].size(); ++j) T[i][j] -= T[i - 2][j];
  }
  auto binom = [](int n, int k) {
    double r = 1.0;
    for (int i = 1; i <= k; ++i) r = r * (n - k + i) / i;
    return r;
  };
  const double s = (b + a) / (b - a), g = -2.0 / (b - a);
  const std::vector<double> &t = T[m + 1];
  double Ts = 0.0;
  for (int kk = 0; kk <= m + 1; ++kk) Ts += t[kk] * std::pow(s, kk);
  std::vector<double> Rx(m + 2, 0.0);  // R(X) in powers of X
  for (int kk = 0; kk <= m + 1; ++kk)
    for (int j = 0; j <= kk; ++j) Rx[j] += t[kk] * binom(kk, j) * std::pow(s, kk - j) * std::pow(g, j) / Ts;
  std::vector<double> pX(m + 1);  // p(X) = (1 - R(X)) / X
  for (int j = 1; j <= m + 1; ++j) pX[j - 1] = -Rx[j];
  for (int i = 0; i <= m; ++i) {  // p(1 - B)
    double v = 0.0;
    for (int j = i; j <= m; ++j) v += pX[j] * binom(j, i) * ((i & 1) ? -1.0 : 1.0);
    cB[i] = v;
  }
}

// Chebyshev interval [CG_CHEB_A, 2] of the block-Jacobi-scaled spectrum
// D^-1 A of the 'backslash' preconditioner (kernels_solve.hip, k_cgs).  The
// lower end trades iterations for parity: 0.06 saves 4 % of the iterations
// but moves the 48x64 smoke pair's mean |uv - oracle| from 6.7e-4 to 6.1e-3
// (knob sweep).
#define CG_CHEB_A 0.04
// the robust GNC stages (alpha < 0.5: D^-1 A with more small eigenvalues):
// 0.02 takes 479 instead of 488 CG iterations per 1080p pair (+1.5 %
// pairs/s; profiles/r3q_cheb_robust_ab.log); 0.01 476 (49.72 / 49.83 vs
// 49.25 / 49.35 pairs/s, parity suites green; profiles/r5aa_cheb01_ab.log).
// Offline at 540p (tools/poly_iters.py's operator): 56 / 54 / 52 / 52
// iterations at 0.04 / 0.02 / 0.01 / 0.005; least-squares polynomials of the
// same degree 62-73; an upper end below 2 makes p negative on the spectrum
#ifndef CG_CHEB_A_ROBUST
#define CG_CHEB_A_ROBUST 0.01
#endif

// Launch geometry of the fused CG iteration kernels for an H x W level.
// k_cg ('pcg'): strips of PCG_SW columns x bands of R rows, 4 bands (waves)
// per 256-thread block, ~CG_PCG_WAVES (640) waves per launch.  k_cgs ('backslash'): strips
// of PCG_SWP columns x bands of R rows, one band per block, ~512 blocks (2
// per CU).  Every block writes one slot of the partials buffer, so the grid
// may not exceed PCG_MAX_BLOCKS blocks: levels wider than PCG_MAX_BLOCKS
// strips are refused (OF_ENOTSUP), never silently mis-sized.
// k_cgs blocks per launch: 2 per CU (LDS-bound) on 256 CUs
#ifndef CGS_TARGET_BLOCKS
#define CGS_TARGET_BLOCKS PCG_MAX_BLOCKS
#endif
// fewest rows per k_cgs band (coarse levels, where the band count is not
// capped by CGS_TARGET_BLOCKS): a launch walks R + 19 row steps
#ifndef CGS_MIN_R
#define CGS_MIN_R 8
#endif
// k_cgs blocks of a fine solve in lanes mode, where OF_TOKEN_SLOTS (2) fine
// solves of different pairs run side by side: one block per CU each, so a
// band is twice as tall (R = 78 at 1080p) and walks R + 19 row steps for R
// rows instead of 39 + 19 (the band halo is recomputed once per band).
// Measured (round 3, 2 x 2 reps): 1 slot x 504 blocks 38.9, 2 x 504 40.7,
// 2 x 336 42.8, 2 x 252 44.4 (4 lanes: 45.3), 2 x 200 42.9, 3 x 168 45.0,
// 4 x 128 42.6 pairs/s (profiles/r3y_token_slots_ab.log, r3z_ab.log); 2 x 270
// (15 bands) 42.2, 3 x 252 44.3 vs 44.8 (profiles/r3ak_ab.log)
#ifndef CGS_LANES_BLOCKS
#define CGS_LANES_BLOCKS 252
#endif
// ... of a fine solve below 1.5 Mpx (864 x 1536, stage 2's first level):
// 168 / 196 / 336 measured 43.6 / 44.0 / 43.6 vs 44.9 pairs/s at 252
// (profiles/r3af_864_blocks_ab.log)
#ifndef CGS_LANES_BLOCKS_S
#define CGS_LANES_BLOCKS_S CGS_LANES_BLOCKS
#endif
// k_cgs blocks of the other (coarse) solves in lanes mode: 128 / 252 measured
// +1 % (45.3 / 45.2 vs 44.8 pairs/s, profiles/r3aa_coarse_blocks_ab.log) but
// would make batches of sub-Mpx pairs differ from estimate_flow; kept at 504
#ifndef CGS_LANES_COARSE_BLOCKS
#define CGS_LANES_COARSE_BLOCKS CGS_TARGET_BLOCKS
#endif
// k_cg waves per launch: config 3 (Classic-C + 'pcg', 720p, 4 lanes) 8.5 /
// 9.45 / 9.73 / 9.42 / 8.10 / 7.40 pairs/s at 256 / 384 / 512 / 768 / 1536 /
// 2048 (profiles/r5au_pcg_waves_ab.log, r5av_pcg_waves_ab.log): shorter
// bands lose to their halo rows and to the lanes' shared CUs; with the
// XCD-aware tile order 10.43 / 10.57 / 10.32 at 512 / 640 / 768
// (profiles/r5ba_pcg_waves_xcd_ab.log)
#ifndef CG_PCG_WAVES
#define CG_PCG_WAVES 640
#endif
int cg_geometry(int H, int W, bool split, of_cg_geometry *g, int target_blocks = CGS_TARGET_BLOCKS) {
  if (H < 1 || W < 1) return OF_EINVAL;
  const int sw = split ? PCG_SWP : PCG_SW;
  const int nstrips = (W + sw - 1) / sw;
  if (nstrips > PCG_MAX_BLOCKS) return OF_ENOTSUP;
  int nbands, R, gy;
  if (split) {
    nbands = std::max(1, std::min((H + CGS_MIN_R - 1) / CGS_MIN_R, target_blocks / nstrips));
    R = (H + nbands - 1) / nbands;
    nbands = (H + R - 1) / R;
    gy = nbands;
  } else {
    nbands = std::max(1, std::min((H + 3) / 4, CG_PCG_WAVES / nstrips));
    R = (H + nbands - 1) / nbands;
    nbands = (H + R - 1) / R;
    gy = (nbands + 3) / 4;
    while (nstrips * gy > PCG_MAX_BLOCKS) {  // ends: gy = 1 once R >= H / 4
      ++R;
      nbands = (H + R - 1) / R;
      gy = (nbands + 3) / 4;
    }
  }
  g->grid_x = nstrips;
  g->grid_y = gy;
  g->rows = R;
  g->bands = nbands;
  g->blocks = nstrips * gy;
  g->strip_cols = sw;
  return g->blocks <= PCG_MAX_BLOCKS ? OF_OK : OF_ENOTSUP;
}

// 'backslash' residual-replacement offers (k_cg_update): before CG launch k
// for k = CG_UPD_FIRST, CG_UPD_FIRST + CG_UPD_EVERY, ... until one acted.
// Solves shorter than CG_UPD_FIRST iterations (the quadratic GNC stage) get
// none: their recursive residual drifts by < 1 % (solve log).
#define CG_UPD_FIRST 16
#define CG_UPD_EVERY 8

// fp64 true residual ||b - A (x [+ x_hi])||^2 and ||b||^2 into out[0..1]
// (solve log)
void log_resid(of_ctx *c, const Img &coef, const F2 &b, const F2 &x, const F2 *xh, double *out) {
  Grid2 g = grid2(b.H, b.W, PCG_MAX_BLOCKS);
  launch(c, "resid", k_resid_part, g.grid, g.block, 0, (const float *)coef.p, coef.ps(), (const float2 *)b.p,
         (const float2 *)x.p, xh ? (const float2 *)xh->p : nullptr, (const PcgState *)(xh ? c->d_state : nullptr),
         b.H, b.W, b.P, c->d_rpart);
  launch(c, "resid", k_resid_final, dim3(1), dim3(OF_BX, OF_BY), 0, (const double *)c->d_rpart, g.nblocks, out);
}

// end of a 'backslash' CG solve: with the solve log on, the true residual of
// the solver's iterate x_hi + x_lo (fp64 sum); then x = fl32(x_hi + x_lo)
void finish_backslash(of_ctx *c, const Img &coef, const F2 &b, const F2 &x, const F2 &xh) {
  if (c->slog_idx >= 0) {
    log_resid(c, coef, b, x, &xh, c->d_rlog + 4 * c->slog_idx);
    c->slog_iter = true;
  }
  Grid2 g = grid2(x.H, x.W);
  launch(c, "cg_finalize", k_cg_finalize, g.grid, g.block, 0, x.p, (const float2 *)xh.p, (const PcgState *)c->d_state,
         x.H, x.W, x.P);
}

SolveResult solve_impl(of_ctx *c, const of_params *P, const Img &coef, const F2 &b, const F2 &x) {
  const int H = b.H, W = b.W;
  c->cur_px = (double)H * W;
  const size_t ps = coef.ps();
  const int solver = P->solver;
  if (solver == OF_SOLVER_PCG || solver == OF_SOLVER_BACKSLASH) {
    const bool block = solver == OF_SOLVER_BACKSLASH;
    float poly[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (block) {
      double cb[CG_DEG + 1];
      cheb_poly(CG_DEG, P->alpha < 0.5 ? CG_CHEB_A_ROBUST : CG_CHEB_A, 2.0, cb);
      for (int i = 0; i <= CG_DEG; ++i) poly[i] = (float)cb[i];
    }
    // ring slot of this solve; a slot is reused only after a synchronisation
    // has drained its previous solve
    if ((int)c->pend.size() >= OF_SOLVE_RING - 1) {
      HIPCHK(hipStreamSynchronize(c->stream));
      drain_solves(c);
    }
    const int slot = c->ring_next;
    c->ring_next = (slot + 1) % OF_SOLVE_RING;
    SolveResult res{0, 0, 0.0};
    res.slot = slot;
    res.px = (double)H * W;
    // 'backslash': one residual replacement at ||r|| < sqrt(rtol) ||b||
    // (k_cg_update), x_hi beside the solve's x
    const double rtol = block ? P->exact_rtol : P->pcg_rtol;
    const double upd_rel = block && rtol > 0 ? std::sqrt(rtol) : 0.0;
    const F2 xh = block ? new_f2(c, H, W) : F2{};
    // coarse levels: the whole solve in one workgroup (k_cg_small)
    if ((double)H * W <= CG_SMALL_PX) {
      CgSmallArgs a;
      a.coef = coef.p;
      a.ps = ps;
      a.b = b.p;
      a.x = x.p;
      a.r = new_f2(c, H, W).p;
      a.p = new_f2(c, H, W).p;
      a.q = new_f2(c, H, W).p;
      a.y = new_f2(c, H, W).p;
      a.t = new_f2(c, H, W).p;
      a.H = H;
      a.W = W;
      a.P = b.P;
      a.rtol = block ? P->exact_rtol : P->pcg_rtol;
      a.maxiter = block ? P->exact_maxiter : P->pcg_maxiter;
      for (int i = 0; i < 8; ++i) a.poly[i] = poly[i];
      a.st = c->d_state;
      a.xh = xh.p;
      a.upd_rel = upd_rel;
      if ((double)H * W <= CG_REG_PX)
        launch(c, "pcg_small", block ? k_cg_reg<CG_DEG, true> : k_cg_reg<0, false>, dim3(1), dim3(64, CGR_T / 64), 0,
               a);
      else
        launch(c, "pcg_small", block ? k_cg_small<CG_DEG, true> : k_cg_small<0, false>, dim3(1), dim3(CGS_BX, CGS_BY),
               0, a);
      if (block) finish_backslash(c, coef, b, x, xh);
      HIPCHK(hipMemcpyAsync(&c->h_ring[slot], c->d_state, sizeof(PcgState), hipMemcpyDeviceToHost, c->stream));
      return res;
    }
    res.name = "pcg_iter";
    // 'backslash': k_cgs (the degree-5 iteration with its stages split over a
    // block's 4 waves); 'pcg': scipy's Jacobi CG in k_cg
    const bool split = block;
    of_cg_geometry geo;
    const bool lanes_fine = c->big && (double)H * W >= c->big_px;  // a token-holding solve
    const int lanes_target = (double)H * W >= 1.5 * (1 << 20) ? CGS_LANES_BLOCKS : CGS_LANES_BLOCKS_S;
    const int gst = cg_geometry(H, W, split, &geo,
                                lanes_fine ? lanes_target : c->big ? CGS_LANES_COARSE_BLOCKS : CGS_TARGET_BLOCKS);
    REQUIRE(gst == OF_OK, gst, "level too wide for the fused CG kernels");
    REQUIRE(coef.ps() * 7 * 4 < 0x40000000ull, OF_ENOTSUP, "level too large for the CG kernels");
    const dim3 grid(geo.grid_x, geo.grid_y), blk(OF_BX, OF_BY);
    const int R = geo.rows, nbands = geo.bands;
    PcgArgs a;
    memset(&a, 0, sizeof(a));
    a.coef = coef.p;
    a.x = x.p;
    a.b = b.p;
    F2 rb[2] = {new_f2(c, H, W), new_f2(c, H, W)}, pb[2] = {new_f2(c, H, W), new_f2(c, H, W)};
    a.H = H;
    a.W = W;
    a.P = b.P;
    a.ps = ps;
    a.nb = geo.blocks;
    a.st = c->d_state;
    a.rtol = rtol;
    a.maxiter = block ? P->exact_maxiter : P->pcg_maxiter;
    a.xh = xh.p;
    a.upd_rel = upd_rel;
    HIPCHK(hipMemsetAsync(c->d_state, 0, sizeof(PcgState), c->stream));
    auto args_k = [&](int k) {
      PcgArgs ak = a;
      const int cur = k & 1, prev = cur ^ 1;
      ak.r_in = rb[prev].p;
      ak.p_old = pb[prev].p;
      ak.r_out = rb[cur].p;
      ak.p_new = pb[cur].p;
      ak.part_rd = c->d_partials + (size_t)prev * 5 * PCG_MAX_BLOCKS;
      ak.part_wr = c->d_partials + (size_t)cur * 5 * PCG_MAX_BLOCKS;
      return ak;
    };
    for (int i = 0; i < 8; ++i) a.poly[i] = poly[i];
    a.hflag = c->d_flag + slot;
    volatile CgFlag *hf = c->h_flag + slot;
    const int enq = run_fed(c, hf, a.maxiter + 1, 3, [&](int k) {
      // the replacement is offered every CG_UPD_EVERY launches until the
      // host sees that it ran (it acts at most once; extra offers are no-ops)
      if (upd_rel > 0 && k >= CG_UPD_FIRST && (k - CG_UPD_FIRST) % CG_UPD_EVERY == 0 && !hf->upd)
        launch(c, "cg_update", k_cg_update, grid, blk, 0, args_k(k), k);
      const bool odd = W & 1;
      auto kern = split ? (k == 0 ? (odd ? k_cgs<true, true> : k_cgs<true, false>)
                                  : (odd ? k_cgs<false, true> : k_cgs<false, false>))
                        : (k == 0 ? (odd ? k_cg<true, false, true> : k_cg<true, false, false>)
                                  : (odd ? k_cg<false, false, true> : k_cg<false, false, false>));
      launch(c, "pcg_iter", kern, grid, blk, 0, args_k(k), k, R, nbands);
    });
    // the convergence test of the last enqueued iterate when the solve ran
    // out of launches (a no-op, skipped, once a prologue declared it done)
    if (!hf->done) launch(c, "pcg_check", k_pcg_check, dim3(1), blk, 0, args_k(enq), enq);
    if (block) finish_backslash(c, coef, b, x, xh);
    HIPCHK(hipMemcpyAsync(&c->h_ring[slot], c->d_state, sizeof(PcgState), hipMemcpyDeviceToHost, c->stream));
    return res;
  }
  // lexicographic SOR (base.py:138-172): 64-row strips of the u half then of
  // the v half (kernels_solve.hip); k_sor_pipe runs many sweeps in flight in
  // one persistent launch, k_sor_lex one launch per sweep (of_set_option
  // OF_OPT_SOR_PIPELINE 0; the same iterate bitwise)
  REQUIRE(solver == OF_SOLVER_SOR, OF_EINVAL, "Unknown solver");
  const int nstrips = (H + 63) / 64;
  REQUIRE(nstrips <= SOR_MAXS, OF_ENOTSUP, "level too tall for the SOR kernel");
  REQUIRE(((double)P->sor_max_iters + 2.0) * (W + 64.0) < 2.0e9, OF_ENOTSUP, "sor_max_iters too large");
  SorArgs a;
  memset(&a, 0, sizeof(a));
  a.coef = coef.p;
  a.b = b.p;
  a.x = x.p;
  a.H = H;
  a.W = W;
  a.P = b.P;
  a.ps = ps;
  a.nstrips = nstrips;
  a.stride = W + 64;
  a.ticket = c->d_sor_sync;
  a.prog = (int *)(c->d_sor_sync + 64);
  a.fail = (int *)(c->d_sor_sync + 32);
  a.st = c->d_state;
  a.omega = (float)P->sor_omega;
  a.tol = P->sor_tol;
  a.maxiter = P->sor_max_iters;
  HIPCHK(hipMemsetAsync(c->d_sor_sync, 0, OF_SOR_SYNC_BYTES, c->stream));
  launch(c, "sor_init", k_sor_init, dim3(std::min(1024, (H * b.P + 63) / 64)), dim3(64), 0, a);
  // levels of <= 64 rows whose sweep ring fits in LDS (OF_OPT_SOR_PIPELINE 2):
  // the pipelined solve in one workgroup, hand-offs through LDS (k_sor_wg)
  if (c->opt_sor_pipe == 2 && a.maxiter > 0 && H <= 64) {
    const size_t buf = sizeof(float2) * (size_t)H * W;
    const int S = (int)std::min<size_t>(SORW_MAXW, OF_SORW_RING_BYTES / buf);
    if (S >= OF_SORW_MIN_RING) {
      SorWgArgs w;
      memset(&w, 0, sizeof(w));
      w.coef = coef.p;
      w.b = b.p;
      w.x = x.p;
      w.H = H;
      w.W = W;
      w.P = b.P;
      w.ps = ps;
      w.S = S;
      w.nw = std::min(SORW_MAXW, 2 * S);
      w.omega = (float)P->sor_omega;
      w.tol = P->sor_tol;
      w.maxiter = P->sor_max_iters;
      w.st = c->d_state;
      w.fail = a.fail;
      launch(c, "sor_wg", k_sor_wg, dim3(1), dim3(64 * w.nw), buf * S + sizeof(SorWgShared), w);
      HIPCHK(hipMemcpyAsync(&c->h_state[0], c->d_state, sizeof(PcgState), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipMemcpyAsync(c->h_norm, a.fail, sizeof(int), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
      if (*(const int *)c->h_norm == 0) {
        const PcgState &st = c->h_state[0];
        REQUIRE(st.done != 0, OF_EHIP, "SOR workgroup solve ended without a decided sweep");
        note_active(c, "sor_wg", st.iter, (double)H * W);
        return {st.iter, st.done, st.xnorm2 > 0 ? std::sqrt(st.rr / st.xnorm2) : 0.0};
      }
      // a wait gave up: x and the state are k_sor_init's; the pipelined
      // kernels below redo the solve (the same iterate)
      ++c->sor_fallbacks;
      HIPCHK(hipMemsetAsync(c->d_sor_sync, 0, OF_SOR_SYNC_BYTES, c->stream));
    }
  }
  if (c->opt_sor_pipe >= 1 && a.maxiter > 0) {
    // ring of S sweep buffers: enough for the sweeps the persistent grid (one
    // wave per CU) can hold in flight, 2 * nstrips units per sweep
    const int S = std::max(4, std::min(SOR_RING_MAX, OF_SOR_PIPE_WAVES / (2 * nstrips) + 2));
    if (!c->d_sorp) HIPCHK(hipMalloc(&c->d_sorp, OF_SORP_BYTES));
    SorPipeArgs q;
    memset(&q, 0, sizeof(q));
    q.coef = coef.p;
    q.b = b.p;
    q.x0 = x.p;
    q.bstride = (size_t)H * b.P;
    const size_t ring_bytes = sizeof(float2) * q.bstride * S;
    if (ring_bytes > c->sor_ring_cap) {
      if (c->d_sor_ring) HIPCHK(hipFree(c->d_sor_ring));
      c->d_sor_ring = nullptr;
      c->sor_ring_cap = 0;
      HIPCHK(hipMalloc(&c->d_sor_ring, ring_bytes));
      c->sor_ring_cap = ring_bytes;
    }
    q.ring = c->d_sor_ring;
    q.H = H;
    q.W = W;
    q.P = b.P;
    q.ps = ps;
    q.nstrips = nstrips;
    q.S = S;
    q.stride = W + 64;
    char *z = c->d_sorp;
    q.ticket = (unsigned *)z;
    q.fail = (int *)(z + 64);
    q.stop = (int *)(z + 128);
    q.cnt = (int *)(z + 256);
    q.dec = (int *)(z + 512);
    q.prog = (int *)(z + 1024);
    q.part = (double *)(z + OF_SORP_SYNC_BYTES);
    q.res = q.part + (size_t)SOR_RING_MAX * 2 * SOR_MAXS * 2;
    q.omega = (float)P->sor_omega;
    q.tol = P->sor_tol;
    q.maxiter = P->sor_max_iters;
    HIPCHK(hipMemsetAsync(z, 0, OF_SORP_SYNC_BYTES, c->stream));
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)q.stop, 0x7fffffff, 1, c->stream));
    // enough waves for S sweeps in flight (more would only poll)
    const int nwaves =
        (int)std::min<int64_t>(std::min(OF_SOR_PIPE_WAVES, 2 * nstrips * S), (int64_t)a.maxiter * 2 * nstrips);
    launch(c, "sor_pipe", k_sor_pipe, dim3(nwaves), dim3(64), OF_SOR_PIPE_SHM, q);
    Grid2 g = grid2(H, W);
    launch(c, "sor_final", k_sor_pipe_final, g.grid, g.block, 0, q, x.p, c->d_state);
    HIPCHK(hipMemcpyAsync(&c->h_state[0], c->d_state, sizeof(PcgState), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(c->h_norm, q.fail, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (*(const int *)c->h_norm == 0) {
      const PcgState &st = c->h_state[0];
      REQUIRE(st.done != 0, OF_EHIP, "SOR pipeline ended without a decided sweep");
      note_active(c, "sor_pipe", st.iter, (double)H * W);
      return {st.iter, st.done, st.xnorm2 > 0 ? std::sqrt(st.rr / st.xnorm2) : 0.0};
    }
    // a hand-off wait timed out (e.g. the grid could not stay resident beside
    // other lanes' work): k_sor_pipe_final left x = 0 and the state as
    // k_sor_init set it, so the per-sweep kernel below redoes the solve from
    // the start (the same iterate and sweep count bitwise)
    ++c->sor_fallbacks;
  }
  double *sor_part = c->d_partials + 10 * PCG_MAX_BLOCKS;  // 2 x [2 * nstrips][2]
  auto args_k = [&](int k) {
    SorArgs ak = a;
    ak.part_rd = sor_part + (size_t)((k + 1) & 1) * 2 * PCG_MAX_BLOCKS;
    ak.part_wr = sor_part + (size_t)(k & 1) * 2 * PCG_MAX_BLOCKS;
    return ak;
  };
  int &hint = iter_hint(c, H, W, solver);
  const int enq = run_chunked(c, a.maxiter, hint > 0 ? std::max(16, hint * 3 / 4) : 16, 64, [&](int k) {
    launch(c, "sor_sweep", k_sor_lex, dim3(2 * nstrips), dim3(64), OF_SOR_SHM, args_k(k), k);
  });
  launch(c, "sor_final", k_sor_final, dim3(1), dim3(64), 0, args_k(enq), enq);
  HIPCHK(hipMemcpyAsync(&c->h_state[0], c->d_state, sizeof(PcgState), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(c->h_norm, a.fail, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  REQUIRE(*(const int *)c->h_norm == 0, OF_EHIP, "SOR strip hand-off timed out");
  const PcgState &st = c->h_state[0];
  hint = st.iter;
  return {st.iter, st.done, st.xnorm2 > 0 ? std::sqrt(st.rr / st.xnorm2) : 0.0};
}

// _solve_linear_system; with the solve log on, followed by the fp64 true
// residual of the final x (diagnostic, off by default)
SolveResult solve(of_ctx *c, const of_params *P, const Img &coef, const F2 &b, const F2 &x) {
  const int idx = c->slog && c->slog_rec.size() < OF_SLOG_MAX ? (int)c->slog_rec.size() : -1;
  c->slog_idx = idx;
  c->slog_iter = false;
  const SolveResult r = solve_impl(c, P, coef, b, x);
  c->slog_idx = -1;
  if (idx >= 0) {
    // residual of the returned fp32 x; also the iterate's unless the solver
    // logged that itself (finish_backslash)
    log_resid(c, coef, b, x, nullptr, c->d_rlog + 4 * idx + 2);
    if (!c->slog_iter) log_resid(c, coef, b, x, nullptr, c->d_rlog + 4 * idx);
    c->slog_rec.push_back({b.H, b.W, P->solver, r.slot, r.iters, r.done, r.rel});
  }
  return r;
}

void note_solve_now(of_stats *st, const SolveResult &r) {
  if (!st) return;
  st->solves++;
  st->solver_iters_total += r.iters;
  st->solver_iters_max = std::max(st->solver_iters_max, r.iters);
  if (r.done == 2) st->solves_not_converged++;
}

// the final state of a deferred CG solve (valid after a stream sync)
SolveResult resolved(of_ctx *c, int slot) {
  const PcgState &s = c->h_ring[slot];
  return {s.iter, s.done, s.bnorm > 0 ? std::sqrt(s.rr) / s.bnorm : 0.0};
}

// statistics of the CG solves since the last stream synchronisation (call
// only after one)
void drain_solves(of_ctx *c) {
  for (auto &l : c->slog_rec)
    if (l.slot >= 0) {
      const SolveResult r = resolved(c, l.slot);
      l.iters = r.iters;
      l.done = r.done;
      l.est = r.rel;
      l.slot = -1;
    }
  for (const auto &p : c->pend) {
    const SolveResult r = resolved(c, p.slot);
    note_solve_now(p.st, r);
    if (p.name) note_active(c, p.name, r.iters + 1, p.px);
  }
  c->pend.clear();
}

void note_solve(of_ctx *c, of_stats *st, const SolveResult &r) {
  if (r.slot >= 0) c->pend.push_back({r.slot, r.px, st, r.name});
  else note_solve_now(st, r);
}

double norm2(of_ctx *c, const F2 &x) {
  Grid2 g = grid2(x.H, x.W, PCG_MAX_BLOCKS);
  launch(c, "norm2", k_norm2_part, g.grid, g.block, 0, (const float2 *)x.p, x.H, x.W, x.P, c->d_partials);
  launch(c, "norm2", k_norm2_final, dim3(1), dim3(OF_BX, OF_BY), 0, (const double *)c->d_partials, g.nblocks,
         c->d_norm);
  HIPCHK(hipMemcpyAsync(c->h_norm, c->d_norm, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  drain_solves(c);
  return *c->h_norm;
}

void median2(of_ctx *c, const F2 &in, const F2 &out, int size) {
  Grid2 g = grid2(in.H, in.W);
  if (size == 5)
    launch(c, "median5", k_median2<5>, g.grid, g.block, 0, (const float2 *)in.p, out.p, in.H, in.W, in.P);
  else if (size == 3)
    launch(c, "median3", k_median2<3>, g.grid, g.block, 0, (const float2 *)in.p, out.p, in.H, in.W, in.P);
  else if (size == 7)
    launch(c, "median7", k_median2<7>, g.grid, g.block, 0, (const float2 *)in.p, out.p, in.H, in.W, in.P);
  else
    throw OfError{OF_ENOTSUP, "median_filter_size must be 3, 5 or 7"};
}

// out = weighted median of uv; with base: out = base + (median - base)
// (classic_nl.py:271-275's uv0 + (filtered - uv0), fused; out may be base)
void wmf(of_ctx *c, const F2 &uv, const Img &guide, const float *occ, const F2 &out, int hsz, double sigma_i,
         const float2 *base = nullptr) {
  REQUIRE(guide.C == 1 || guide.C == 3, OF_ENOTSUP, "weighted median guide must have 1 or 3 channels");
  REQUIRE(hsz >= 0 && hsz <= 12, OF_ENOTSUP, "area_hsz must be <= 12");
  const int RW = WMF_T + 2 * hsz, nreg = RW * RW;
  const int RP = RW + ((8 - RW) % 16 + 16) % 16;  // record row pitch, RP % 16 == 8 (conflict-free window reads)
  int npow2 = 64;
  while (npow2 < nreg) npow2 <<= 1;
  const int nper = npow2 / 64;  // sort keys per lane: 1..16
  const size_t shm = 2 * (size_t)wmf_nc(npow2) * 64 * sizeof(wmf_sum_t) + (size_t)RW * RP * (guide.C == 3 ? 16 : 8) +
                     2 * (size_t)npow2 * sizeof(uint16_t) + 2 * (size_t)RW * RP;
  dim3 grid((uv.W + WMF_T - 1) / WMF_T, (uv.H + WMF_T - 1) / WMF_T);
  const float nk = (float)(-1.4426950408889634 / (2.0 * sigma_i * sigma_i));  // -log2(e) / (2 sigma^2)
  const dim3 block(64);
  auto pick = [&](auto k1, auto k2, auto k4, auto k8, auto k8h7, auto k16) {
    auto k = nper == 1 ? k1 : nper == 2 ? k2 : nper == 4 ? k4 : nper == 8 ? (hsz == 7 ? k8h7 : k8) : k16;
    launch(c, "wmf", k, grid, block, shm, (const float2 *)uv.p, (const float *)guide.p, occ, out.p, uv.H, uv.W,
           uv.P, guide.ps(), hsz, nk, RW, RP, base);
  };
  if (guide.C == 3)
    pick(k_wmf<3, 1, 0>, k_wmf<3, 2, 0>, k_wmf<3, 4, 0>, k_wmf<3, 8, 0>, k_wmf<3, 8, 7>, k_wmf<3, 16, 0>);
  else
    pick(k_wmf<1, 1, 0>, k_wmf<1, 2, 0>, k_wmf<1, 4, 0>, k_wmf<1, 8, 0>, k_wmf<1, 8, 7>, k_wmf<1, 16, 0>);
}

void resample_f2(of_ctx *c, const F2 &in, const F2 &out) {
  const float ratio = (float)((double)out.H / (double)in.H);
  Grid2 g = grid2(out.H, out.W);
  launch(c, "resample_flow", k_resize<float2>, g.grid, g.block, 0, (const float2 *)in.p, in.H, in.W, in.P,
         (size_t)in.H * in.P, out.p, out.H, out.W, out.P, (size_t)out.H * out.P, ratio);
}

// ---- the per-level IRLS loops ----------------------------------------------
struct LevelIn {
  Img im;     // 2*nc planes
  Img guide;  // gc planes or p == nullptr
};

// Lanes mode (of_pairs_run, of_pairs_run_host): every linear solve on a
// level of >= big_px pixels (solve_tok below) holds one of the lanes' token
// slots (OF_TOKEN_SLOTS = 2) until its GPU work has drained, and runs its
// k_cgs launches with CGS_LANES_BLOCKS (252, one per CU) blocks, so two fine
// solves of different pairs fill the chip side by side with bands twice as
// tall as one solve's 504 blocks would have.  Until round 3 the token had one
// slot and a fine solve 504 blocks (two lanes' 504-block launches
// interleaving at block granularity stall each other: 2 slots x 504 blocks is
// only +4 %).  Warps, assembly and the weighted median of fine levels run
// unserialised.  Tried and rejected (round 3): the token
// holder's solve on a shared high-priority stream, 32.3-32.8 vs 35.5-36.2
// pairs/s (profiles/r3f_cg_priority_ab.log).  Outside lanes mode: no-op.
// The full-size preprocessing (ROF, pyramids) ran under the token through
// round 3; without it (A/B, 2 x 2 reps): 39.02 vs 38.40 pairs/s host to
// host, bitwise the same flows (profiles/r3u_ab.log, r3v_ab.log)
#ifndef OF_PRE_TOKEN
#define OF_PRE_TOKEN 0
#endif
struct BigPhase {
  of_ctx *c;
  bool held = false;
  BigPhase(of_ctx *c_, double px) : c(c_) {
    if (c->big && px >= c->big_px) {
      c->big->lock();
      held = true;
    }
  }
  ~BigPhase() {
    if (held) {
      hipStreamSynchronize(c->stream);
      c->big->unlock();
    }
  }
};

// Only the fine solves hold the token: a fine level's assembly, warps and
// weighted median (VALU/LDS-bound) overlap another lane's CG (issue- and
// HBM-bound); measured 33.8 -> 34.5 pairs/s at 3 lanes vs holding the token
// through whole fine levels
// OF_SOLVE_PRIO: a token-holding solve runs on its lane's high-priority
// stream, so its blocks are dispatched ahead of other lanes' kernels as CUs
// free up (a 252-block k_cgs launch needs 74 KB of LDS per CU, which the
// weighted median's 19 KB waves otherwise keep refilling: in the default
// bench's trace the first launch of a 1080p fine solve takes 92 us median but
// 851 us at p90).  Measured with the side-by-side solves: 42.0-43.1 vs
// 45.0-45.2 pairs/s (3 reps, profiles/r3ai_solve_prio_ab.log), as round 3's
// single-slot version was (-10 %): starving the other lanes costs more than
// the CG gains.  Off.
#ifndef OF_SOLVE_PRIO
#define OF_SOLVE_PRIO 0
#endif
SolveResult solve_tok(of_ctx *c, const of_params *P, const Img &coef, const F2 &b, const F2 &x) {
  BigPhase bp(c, (double)b.H * b.W);
  if (!(OF_SOLVE_PRIO && bp.held)) return solve(c, P, coef, b, x);
  if (!c->hp) {
    int least = 0, greatest = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIPCHK(hipStreamCreateWithPriority(&c->hp, hipStreamNonBlocking, greatest));
    for (auto &e : c->ev_hp) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  HIPCHK(hipEventRecord(c->ev_hp[0], c->stream));
  HIPCHK(hipStreamWaitEvent(c->hp, c->ev_hp[0], 0));
  std::swap(c->stream, c->hp);
  SolveResult r;
  try {
    r = solve(c, P, coef, b, x);
  } catch (...) {
    std::swap(c->stream, c->hp);
    throw;
  }
  std::swap(c->stream, c->hp);
  HIPCHK(hipEventRecord(c->ev_hp[1], c->hp));
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_hp[1], 0));
  return r;
}

// ---- general spatial_filters (kernels_gen.hip) ------------------------------
// radius of the DIA offset grid: filters of fh x fw taps couple pixels up to
// (fh - 1, fw - 1) apart
int gen_radius(const of_params *P) {
  int D = 0;
  for (int q = 0; q < P->filters.n; ++q) D = std::max(D, std::max(P->filters.fh[q], P->filters.fw[q]) - 1);
  return D;
}
int gen_nplanes(int D) { return 2 * (2 * D + 1) * (2 * D + 1) + 1; }

GenFilters gen_filters(const of_params *P) {
  GenFilters f;
  memset(&f, 0, sizeof(f));
  f.n = P->filters.n;
  f.D = gen_radius(P);
  for (int q = 0; q < f.n; ++q) {
    f.fh[q] = P->filters.fh[q];
    f.fw[q] = P->filters.fw[q];
    for (int t = 0; t < f.fh[q] * f.fw[q]; ++t) f.taps[q][t] = (float)P->filters.taps[q][t];
    f.ru[q] = to_penf(P->filters.rho_u[q]);
    f.rv[q] = to_penf(P->filters.rho_v[q]);
    f.qu[q] = to_penf(P->filters.qua_u[q]);
    f.qv[q] = to_penf(P->filters.qua_v[q]);
  }
  return f;
}

// per-level buffers of the general path: filter weights, DIA planes, CG vectors
struct GenLevel {
  int D = 0;
  Img w, pl;
  F2 r, p, z, q, t, e;
};
GenLevel gen_level(of_ctx *c, const of_params *P, int H, int W) {
  GenLevel L;
  L.D = gen_radius(P);
  L.w = new_img(c, H, W, std::max(1, 2 * P->filters.n));
  L.pl = new_img(c, H, W, gen_nplanes(L.D));
  L.r = new_f2(c, H, W);
  L.p = new_f2(c, H, W);
  L.z = new_f2(c, H, W);
  L.q = new_f2(c, H, W);
  L.t = new_f2(c, H, W);
  L.e = new_f2(c, H, W);
  return L;
}

void gen_flow_operator(of_ctx *c, const of_params *P, const OpArgs &o, const F2 &uv, const F2 *duv, const Img &It,
                       const Img &Ix, const Img &Iy, const F2 *uvhat, const GenLevel &L, const F2 &rhs) {
  const GenFilters f = gen_filters(P);
  Grid2 g = grid2(uv.H, uv.W);
  if (f.n)
    launch(c, "gen_weights", k_gen_weights, g.grid, g.block, 0, f, o, (const float2 *)uv.p,
           (const float2 *)(duv ? duv->p : nullptr), uv.H, uv.W, uv.P, L.w.ps(), L.w.p);
  launch(c, "gen_dia", k_gen_dia, g.grid, g.block, 0, f, o, (const float *)L.w.p, (const float2 *)uv.p,
         (const float2 *)(duv ? duv->p : nullptr), (const float *)It.p, (const float *)Ix.p, (const float *)Iy.p, It.C,
         (const float2 *)(uvhat ? uvhat->p : nullptr), uv.H, uv.W, uv.P, L.pl.ps(), L.pl.p, rhs.p);
}

// CG on the DIA operator with the scipy control flow from x = 0; returns
// (iterations, done)
std::pair<int, int> dia_cg(of_ctx *c, DiaArgs a, int nb, Grid2 g) {
  HIPCHK(hipMemsetAsync(a.st, 0, sizeof(PcgState), c->stream));
  launch(c, "dia_init", k_dia_init, g.grid, g.block, 0, a);
  int it = 0;
  for (;;) {
    const int n = std::min(32, a.maxiter + 1 - it);
    for (int t = 0; t < n; ++t, ++it) {
      launch(c, "dia_dir", k_dia_dir, g.grid, g.block, 0, a, it, nb);
      launch(c, "dia_q", k_dia_q, g.grid, g.block, 0, a, it);
      launch(c, "dia_upd", k_dia_upd, g.grid, g.block, 0, a, it, nb);
    }
    HIPCHK(hipMemcpyAsync(&c->h_state[0], a.st, sizeof(PcgState), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->h_state[0].done || it > a.maxiter) break;
  }
  return {c->h_state[0].iter, c->h_state[0].done};
}

// _solve_linear_system (base.py:87-172) on a DIA operator
SolveResult gen_solve(of_ctx *c, const of_params *P, const GenLevel &L, const F2 &b, const F2 &x) {
  const int H = b.H, W = b.W;
  DiaArgs a;
  memset(&a, 0, sizeof(a));
  a.pl = L.pl.p;
  a.ps = L.pl.ps();
  a.D = L.D;
  a.H = H;
  a.W = W;
  a.P = b.P;
  a.b = b.p;
  a.x = x.p;
  a.r = L.r.p;
  a.p = L.p.p;
  a.z = L.z.p;
  a.q = L.q.p;
  a.part = c->d_partials;
  a.st = c->d_state;
  const size_t vbytes = sizeof(float2) * (size_t)H * b.P;
  if (P->solver == OF_SOLVER_SOR) {
    HIPCHK(hipMemsetAsync(x.p, 0, vbytes, c->stream));
    HIPCHK(hipMemsetAsync(a.st, 0, sizeof(PcgState), c->stream));
    const int nt = std::min(1024, (W + 63) / 64 * 64);
    launch(c, "dia_sor", k_dia_sor, dim3(1), dim3(nt), 0, a, (float)P->sor_omega, P->sor_max_iters, P->sor_tol);
    HIPCHK(hipMemcpyAsync(&c->h_state[0], a.st, sizeof(PcgState), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return {c->h_state[0].iter, c->h_state[0].done, 0.0};
  }
  REQUIRE(P->solver == OF_SOLVER_PCG || P->solver == OF_SOLVER_BACKSLASH, OF_EINVAL, "Unknown solver");
  const bool bs = P->solver == OF_SOLVER_BACKSLASH;
  a.block = bs;
  Grid2 g = grid2(H, W, PCG_MAX_BLOCKS);
  const int nb = g.nblocks;
  // ||b||
  {
    launch(c, "norm2", k_norm2_part, g.grid, g.block, 0, (const float2 *)b.p, H, W, b.P, c->d_partials);
    launch(c, "norm2", k_norm2_final, dim3(1), dim3(OF_BX, OF_BY), 0, (const double *)c->d_partials, nb, c->d_norm);
    HIPCHK(hipMemcpyAsync(c->h_norm, c->d_norm, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  const double bnorm = std::sqrt(*c->h_norm);
  if (!bs) {
    // scipy cg (base.py:116-136): Jacobi, rtol pcg_rtol, maxiter pcg_maxiter
    a.atol = P->pcg_rtol * bnorm;
    a.maxiter = P->pcg_maxiter;
    const auto r = dia_cg(c, a, nb, g);
    return {r.first, r.second, bnorm > 0 ? std::sqrt(c->h_state[0].rr) / bnorm : 0.0};
  }
  // 'backslash' surrogate: 2x2 block-Jacobi CG to exact_rtol, then iterative
  // refinement x += CG(A, b - A x) on the fp64 true residual until it meets
  // exact_rtol ||b|| (at most 4 corrections)
  const double goal = P->exact_rtol * bnorm;
  a.atol = 0.5 * goal;
  a.maxiter = P->exact_maxiter;
  auto r = dia_cg(c, a, nb, g);
  int iters = r.first, done = r.second;
  double rel = 0.0;
  for (int ref = 0;; ++ref) {
    DiaArgs t = a;
    t.x = x.p;
    launch(c, "dia_resid", k_dia_resid, g.grid, g.block, 0, t, L.t.p);
    launch(c, "dia_sum", k_dia_sum, dim3(1), dim3(OF_BX, OF_BY), 0, (const double *)(c->d_partials + 8 * PCG_MAX_BLOCKS),
           nb, c->d_norm);
    HIPCHK(hipMemcpyAsync(c->h_norm, c->d_norm, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const double tn = std::sqrt(*c->h_norm);
    rel = bnorm > 0 ? tn / bnorm : 0.0;
    if (tn <= goal || ref >= 4 || iters >= P->exact_maxiter) break;
    DiaArgs e = a;
    e.b = L.t.p;
    e.x = L.e.p;
    e.maxiter = P->exact_maxiter - iters;
    r = dia_cg(c, e, nb, g);
    iters += r.first;
    done = r.second;
    launch(c, "dia_acc", k_dia_acc, g.grid, g.block, 0, x.p, (const float2 *)L.e.p, H, W, b.P);
  }
  return {iters, rel <= P->exact_rtol ? 1 : done, rel};
}

// gen_solve with the solve log (of_set_solve_log): the fp64 true residual
// ||b - A x|| / ||b|| of the DIA operator (k_dia_resid) for the iterate and
// the returned x (the same fp32 field here)
SolveResult gen_solve_logged(of_ctx *c, const of_params *P, const GenLevel &L, const F2 &b, const F2 &x) {
  const SolveResult r = gen_solve(c, P, L, b, x);
  if (c->slog && c->slog_rec.size() < OF_SLOG_MAX) {
    const int idx = (int)c->slog_rec.size();
    double *out = c->d_rlog + 4 * idx;
    DiaArgs a;
    memset(&a, 0, sizeof(a));
    a.pl = L.pl.p;
    a.ps = L.pl.ps();
    a.D = L.D;
    a.H = b.H;
    a.W = b.W;
    a.P = b.P;
    a.b = b.p;
    a.x = x.p;
    a.part = c->d_partials;
    Grid2 g = grid2(b.H, b.W, PCG_MAX_BLOCKS);
    launch(c, "dia_resid", k_dia_resid, g.grid, g.block, 0, a, L.t.p);
    launch(c, "dia_sum", k_dia_sum, dim3(1), dim3(OF_BX, OF_BY), 0, (const double *)(c->d_partials + 8 * PCG_MAX_BLOCKS),
           g.nblocks, out);
    launch(c, "norm2", k_norm2_part, g.grid, g.block, 0, (const float2 *)b.p, b.H, b.W, b.P, c->d_rpart);
    launch(c, "norm2", k_norm2_final, dim3(1), dim3(OF_BX, OF_BY), 0, (const double *)c->d_rpart, g.nblocks, out + 1);
    HIPCHK(hipMemcpyAsync(out + 2, out, 2 * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    c->slog_rec.push_back({b.H, b.W, P->solver, -1, r.iters, r.done, r.rel});
  }
  return r;
}

// HSOpticalFlow.compute_flow_base (hs.py:109-142)
// ---- progress reports (of_set_progress) ----
struct ProgressOff {  // batch entries: the context (lane 0) does not report
  of_ctx *c;
  of_progress_fn fn;
  explicit ProgressOff(of_ctx *c_) : c(c_), fn(c_->prog_fn) { c->prog_fn = nullptr; }
  ~ProgressOff() { c->prog_fn = fn; }
};
of_progress prog_event(of_ctx *c, int event, int h, int w) {
  of_progress e;
  memset(&e, 0, sizeof(e));
  e.event = event;
  e.stage = c->prog_stage;
  e.level = c->prog_level;
  e.h = h;
  e.w = w;
  return e;
}
// an iteration's solve is done: ||clip(x) - d|| (d may be null) or, with
// limit < 0, ||x|| (HS)
void prog_iter(of_ctx *c, int it, int jl, const F2 &x, const F2 *d, int limit) {
  if (!c->prog_fn) return;
  of_progress e = prog_event(c, OF_EV_ITER, x.H, x.W);
  e.iter = it;
  e.lin = jl;
  e.norm = std::nan("");
  if (c->prog_flags & OF_PROGRESS_ITER) {
    Grid2 g = grid2(x.H, x.W, PCG_MAX_BLOCKS);
    launch(c, "step_norm2", k_step_norm2_part, g.grid, g.block, 0, (const float2 *)x.p,
           d ? (const float2 *)d->p : (const float2 *)nullptr, limit > 0 ? 1 : 0, x.H, x.W, x.P, c->d_partials);
    launch(c, "step_norm2", k_norm2_final, dim3(1), dim3(OF_BX, OF_BY), 0, (const double *)c->d_partials, g.nblocks,
           c->d_norm);
    HIPCHK(hipMemcpyAsync(c->h_norm, c->d_norm, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    drain_solves(c);
    e.norm = std::sqrt(*c->h_norm);
  }
  c->prog_fn(c->prog_user, &e);
}

void hs_base(of_ctx *c, const of_params *P, const LevelIn &L, F2 &uv, of_stats *st) {
  const int H = L.im.H, W = L.im.W, nc = L.im.C / 2;
  c->cur_px = (double)H * W;
  LevelDeriv D = level_deriv(c, L.im, nc, P->interp, P->deriv_filter, 0.5);
  Img It = new_img(c, H, W, nc), Ix = new_img(c, H, W, nc), Iy = new_img(c, H, W, nc);
  Img coef = new_img(c, H, W, 7);
  F2 rhs = new_f2(c, H, W), x = new_f2(c, H, W), tmp = new_f2(c, H, W);
  OpArgs o = op_args(P, 0.0, 0.0);
  Grid2 g = grid2(H, W);
  const bool fuse = can_fuse_warp_op(c, o, nc);
  for (int it = 0; it < P->max_warping_iters; ++it) {
    if (fuse) {
      warp_operator(c, D, P->interp, o, uv, coef, rhs);
    } else {
      partial_deriv(c, D, P->interp, uv, It, Ix, Iy);
      flow_operator(c, o, uv, nullptr, It, Ix, Iy, nullptr, coef, rhs);
    }
    note_solve(c, st, solve_tok(c, P, coef, rhs, x));
    c->cur_px = (double)H * W;
    const double xn = std::sqrt(norm2(c, x));
    if (c->prog_fn) {  // hs.py:123-124 prints ||x|| before the exit test
      of_progress e = prog_event(c, OF_EV_ITER, H, W);
      e.iter = it;
      e.norm = xn;
      c->prog_fn(c->prog_user, &e);
    }
    if (xn < 1e-3) break;
    launch(c, "add_update", k_add_update, g.grid, g.block, 0, uv.p, (const float2 *)x.p, P->limit_update, H, W, uv.P);
    if (P->median_filter_size)
      for (int m = 0; m < P->mf_iter; ++m) {
        median2(c, uv, tmp, P->median_filter_size);
        std::swap(uv.p, tmp.p);
      }
  }
}

// BAOpticalFlow / ClassicNLOpticalFlow compute_flow_base (ba.py:143-206,
// classic_nl.py:200-277)
void irls_base(of_ctx *c, const of_params *P, const LevelIn &L, F2 &uv, double alpha, int max_linear,
               of_stats *st) {
  const int H = L.im.H, W = L.im.W, nc = L.im.C / 2;
  c->cur_px = (double)H * W;
  const double blend = P->method == OF_METHOD_BA ? P->blend : 0.5;  // classic_nl.py:232 passes no blend
  LevelDeriv D = level_deriv(c, L.im, nc, P->interp, P->deriv_filter, blend);
  Img It = new_img(c, H, W, nc), Ix = new_img(c, H, W, nc), Iy = new_img(c, H, W, nc);
  Img coef = new_img(c, H, W, 7);
  Img occ = new_img(c, H, W, 1);
  F2 rhs = new_f2(c, H, W), x = new_f2(c, H, W), uv1 = new_f2(c, H, W), uv2 = new_f2(c, H, W);
  F2 duv = new_f2(c, H, W);
  OpArgs o = op_args(P, alpha, 0.0);
  Grid2 g = grid2(H, W);
  const bool nl = P->method == OF_METHOD_CLASSIC_NL;
  const bool gen = P->filters.general;
  GenLevel GL;
  if (gen) GL = gen_level(c, P, H, W);
  // one linearisation per warp: warp + assembly fused (no derivative planes)
  const bool fuse = !gen && max_linear == 1 && can_fuse_warp_op(c, o, nc);
  for (int it = 0; it < P->max_iters; ++it) {
    if (!fuse) partial_deriv(c, D, P->interp, uv, It, Ix, Iy);
    for (int jl = 0; jl < max_linear; ++jl) {
      if (gen) {
        gen_flow_operator(c, P, o, uv, jl ? &duv : nullptr, It, Ix, Iy, nullptr, GL, rhs);
        note_solve(c, st, gen_solve_logged(c, P, GL, rhs, x));
      } else if (fuse) {
        warp_operator(c, D, P->interp, o, uv, coef, rhs);
        note_solve(c, st, solve_tok(c, P, coef, rhs, x));
      } else {
        flow_operator(c, o, uv, jl ? &duv : nullptr, It, Ix, Iy, nullptr, coef, rhs);
        note_solve(c, st, solve_tok(c, P, coef, rhs, x));
      }
      c->cur_px = (double)H * W;
      prog_iter(c, it, jl, x, jl ? &duv : nullptr, P->limit_update);
      const bool filt = P->median_filter_size != 0;
      launch(c, nl && filt && L.guide.p ? "update_occ" : "update", k_update_occ, g.grid, g.block, 0,
             (const float2 *)uv.p, (const float2 *)x.p, P->limit_update, uv1.p, (const float *)L.im.p,
             (const float *)L.im.plane(nc), nc, (nl && filt && L.guide.p) ? occ.p : (float *)nullptr, H, W, uv.P,
             L.im.ps());
      const bool last = jl + 1 >= max_linear;
      if (last && filt && nl && L.guide.p) {
        // uv = uv0 + (filtered - uv0) (classic_nl.py:271-275) in the weighted
        // median's own store
        wmf(c, uv1, L.guide, occ.p, uv, P->area_hsz, P->sigma_i, (const float2 *)uv.p);
        continue;
      }
      F2 res = uv1;
      if (filt) {
        if (nl && L.guide.p) wmf(c, uv1, L.guide, occ.p, uv2, P->area_hsz, P->sigma_i);
        else median2(c, uv1, uv2, P->median_filter_size);
        res = uv2;
      }
      if (!last)  // duv = filtered - uv feeds the next linearisation
        launch(c, "sub2", k_sub2, g.grid, g.block, 0, (const float2 *)uv.p, (const float2 *)res.p, duv.p, H, W, uv.P);
      else  // uv = uv0 + (filtered - uv0)  (classic_nl.py:271-275, ba.py:404-407)
        launch(c, "axpy_diff", k_axpy_diff, g.grid, g.block, 0, uv.p, (const float2 *)uv.p, (const float2 *)res.p, H,
               W, uv.P);
    }
  }
}

// AltBAOpticalFlow.compute_flow_base (alt_ba.py:189-274)
void altba_base(of_ctx *c, const of_params *P, const LevelIn &L, F2 &uv, F2 &uvhat, double alpha, bool replacement,
                of_stats *st) {
  const int H = L.im.H, W = L.im.W, nc = L.im.C / 2;
  c->cur_px = (double)H * W;
  LevelDeriv D = level_deriv(c, L.im, nc, P->interp, P->deriv_filter, 0.5);
  Img It = new_img(c, H, W, nc), Ix = new_img(c, H, W, nc), Iy = new_img(c, H, W, nc);
  Img coef = new_img(c, H, W, 7);
  F2 rhs = new_f2(c, H, W), x = new_f2(c, H, W), duv = new_f2(c, H, W), t1 = new_f2(c, H, W), t2 = new_f2(c, H, W);
  Grid2 g = grid2(H, W);
  const int n = P->max_iters;
  const bool gen = P->filters.general;
  GenLevel GL;
  if (gen) GL = gen_level(c, P, H, W);
  std::vector<double> l2s(n + 1);
  const double a = std::log10(1e-4), b = std::log10(P->lambda2);
  for (int t = 0; t < n; ++t) l2s[t] = std::pow(10.0, n == 1 ? a : a + (b - a) * t / (n - 1));
  l2s[n] = P->lambda2;
  double lambda2 = l2s[0];
  for (int i = 0; i < n; ++i) {
    partial_deriv(c, D, P->interp, uv, It, Ix, Iy);
    OpArgs o = op_args(P, alpha, lambda2);
    bool have_duv = false;
    for (int jl = 0; jl < P->max_linear; ++jl) {
      if (gen) {
        gen_flow_operator(c, P, o, uv, have_duv ? &duv : nullptr, It, Ix, Iy, &uvhat, GL, rhs);
        note_solve(c, st, gen_solve_logged(c, P, GL, rhs, x));
      } else {
        flow_operator(c, o, uv, have_duv ? &duv : nullptr, It, Ix, Iy, &uvhat, coef, rhs);
        note_solve(c, st, solve_tok(c, P, coef, rhs, x));
      }
      c->cur_px = (double)H * W;
      prog_iter(c, i, jl, x, have_duv ? &duv : nullptr, P->limit_update);
      // duv = clip(x): computed as (0 + clip(x))
      HIPCHK(hipMemsetAsync(duv.p, 0, sizeof(float2) * (size_t)H * duv.P, c->stream));
      launch(c, "add_update", k_add_update, g.grid, g.block, 0, duv.p, (const float2 *)x.p, P->limit_update, H, W,
             duv.P);
      have_duv = true;
    }
    if (have_duv)
      launch(c, "add_update", k_add_update, g.grid, g.block, 0, uv.p, (const float2 *)duv.p, 0, H, W, uv.P);
    // uvhat = denoise_LO(uv) per component (denoising.py:6-30)
    if (P->median_filter_size) {
      HIPCHK(hipMemcpyAsync(t1.p, uv.p, sizeof(float2) * (size_t)H * uv.P, hipMemcpyDeviceToDevice, c->stream));
      const float lam = (float)(lambda2 / P->lambda3);
      for (int k = 0; k < P->itersLO; ++k) {
        launch(c, "lo_blend", k_lo_blend, g.grid, g.block, 0, (const float2 *)t1.p, (const float2 *)uv.p, lam, t2.p, H,
               W, uv.P);
        median2(c, t2, t1, P->median_filter_size);
      }
      HIPCHK(hipMemcpyAsync(uvhat.p, t1.p, sizeof(float2) * (size_t)H * uv.P, hipMemcpyDeviceToDevice, c->stream));
    } else {
      HIPCHK(hipMemcpyAsync(uvhat.p, uv.p, sizeof(float2) * (size_t)H * uv.P, hipMemcpyDeviceToDevice, c->stream));
    }
    if (replacement)
      HIPCHK(hipMemcpyAsync(uv.p, uvhat.p, sizeof(float2) * (size_t)H * uv.P, hipMemcpyDeviceToDevice, c->stream));
    lambda2 = l2s[i + 1];
  }
}

int auto_levels(int H, int W, double spacing) {
  int m = H < W ? H : W;  // base.py:192-195
  return 1 + (int)std::floor(std::log(m / 16.0) / std::log(spacing));
}

void check_params(const of_params *P) {
  REQUIRE(P->method >= 0 && P->method <= 3, OF_EINVAL, "unknown method");
  REQUIRE(P->solver >= 0 && P->solver <= 2, OF_EINVAL, "Unknown solver");
  REQUIRE(P->interp >= 0 && P->interp <= 2, OF_EINVAL, "Unknown interpolation method");
  REQUIRE(P->median_filter_size == 0 || P->median_filter_size == 3 || P->median_filter_size == 5 ||
              P->median_filter_size == 7,
          OF_ENOTSUP, "median_filter_size must be None, 3, 5 or 7");
  if (P->filters.general) {
    REQUIRE(P->filters.n >= 0 && P->filters.n <= OF_MAX_FILTERS, OF_ENOTSUP, "at most 8 spatial filters");
    for (int q = 0; q < P->filters.n; ++q)
      REQUIRE(P->filters.fh[q] >= 1 && P->filters.fh[q] <= OF_MAX_FDIM && P->filters.fw[q] >= 1 &&
                  P->filters.fw[q] <= OF_MAX_FDIM,
              OF_ENOTSUP, "spatial filters of at most 5 x 5 taps");
  }
}

// compute_flow (hs.py:49-99, ba.py:57-138, classic_nl.py:89-198, alt_ba.py:81-187)
// images: device 2nc planes; guide: device gc planes or p == nullptr;
// uv_io: full-resolution flow (init in, result out).
void compute_flow_dev(of_ctx *c, of_params *P, const Img &images, const Img &guide, F2 &uv_io, of_stats *st) {
  check_params(P);
  const int H = images.H, W = images.W, C = images.C, nc = C / 2;
  REQUIRE(nc >= 1 && nc <= OF_MAX_NC, OF_ENOTSUP, "1..4 channels per frame supported");
  hipEvent_t t0 = timing_event(c), t1 = timing_event(c);
  HIPCHK(hipEventRecord(t0, c->stream));
  c->prog_t0 = std::chrono::steady_clock::now();
  // preprocessing (under the lanes' token with OF_PRE_TOKEN)
  std::unique_ptr<BigPhase> pre(new BigPhase(c, OF_PRE_TOKEN ? (double)H * W : 0.0));
  Img img;
  if (P->texture) {
    const double alp = (P->method == OF_METHOD_HS || P->method == OF_METHOD_ALT_BA) ? 0.95 : P->alp;
    img = rof_texture(c, images, 1.0 / 8, 100, alp);
  } else if (P->fc && (P->method == OF_METHOD_BA || P->method == OF_METHOD_CLASSIC_NL)) {
    // images - alp * correlate(images, gaussian(5, 1.5)) then [0, 255]
    // (classic_nl.py:109-113, ba.py:280-285), per channel
    auto gk = gaussian(5, 1.5);
    Img sm = new_img(c, H, W, C);
    correlate(c, images, sm, make_taps(gk.data(), 5, 5));
    img = new_img(c, H, W, C);
    Grid2 g = grid2(H, W);
    launch(c, "sub_scaled", k_sub_scaled, gz(g, C), g.block, 0, (const float *)images.p, (const float *)sm.p,
           (float)P->alp, img.p, H, W, img.P, img.ps());
    scale_img(c, img, 0.0f, 255.0f, 2);
  } else {
    img = new_img(c, H, W, C);
    copy_img(c, img, images);
    scale_img(c, img, 0.0f, 255.0f, 2);
  }
  int levels = P->pyramid_levels;
  if (P->method == OF_METHOD_HS || P->method == OF_METHOD_ALT_BA || P->auto_level)
    levels = auto_levels(H, W, P->pyramid_spacing);
  P->pyramid_levels = levels;
  REQUIRE(levels <= OF_MAX_LEVELS, OF_EINVAL, "too many pyramid levels");
  std::vector<Img> pyr = build_pyramid(c, img, levels, P->pyramid_spacing), gpyr, cpyr, cgpyr;
  if (P->method != OF_METHOD_HS) gpyr = build_pyramid(c, img, P->gnc_pyramid_levels, P->gnc_pyramid_spacing);
  const bool use_guide = P->method == OF_METHOD_CLASSIC_NL && guide.p;
  if (use_guide) {
    cpyr = build_pyramid(c, guide, levels, P->pyramid_spacing);
    cgpyr = build_pyramid(c, guide, P->gnc_pyramid_levels, P->gnc_pyramid_spacing);
  }
  HIPCHK(hipEventRecord(t1, c->stream));
  pre.reset();
  F2 uv = uv_io, uvhat;
  if (P->method == OF_METHOD_ALT_BA) {
    uvhat = new_f2(c, H, W);
    HIPCHK(hipMemcpyAsync(uvhat.p, uv.p, sizeof(float2) * (size_t)H * uv.P, hipMemcpyDeviceToDevice, c->stream));
  }
  const double alpha_orig = P->alpha;
  const int gnc = P->method == OF_METHOD_HS ? 1 : P->gnc_iters;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> lev_ev;
  for (int ig = 0; ig < gnc; ++ig) {
    const int nl = ig == 0 ? levels : P->gnc_pyramid_levels;
    const std::vector<Img> &lv = ig == 0 ? pyr : gpyr;
    c->prog_stage = ig;
    c->prog_level = -1;
    if (c->prog_fn) {
      of_progress e = prog_event(c, OF_EV_STAGE, H, W);
      c->prog_fn(c->prog_user, &e);
    }
    for (int l = nl - 1; l >= 0; --l) {
      const int h = lv[l].H, w = lv[l].W;
      c->prog_level = l;
      if (c->prog_fn) {
        of_progress e = prog_event(c, OF_EV_LEVEL, h, w);
        c->prog_fn(c->prog_user, &e);
      }
      hipEvent_t e0 = timing_event(c), e1 = timing_event(c);
      HIPCHK(hipEventRecord(e0, c->stream));
      if (uv.H != h || uv.W != w) {
        F2 nuv = new_f2(c, h, w);
        resample_f2(c, uv, nuv);
        uv = nuv;
        if (uvhat.p) {
          F2 nh = new_f2(c, h, w);
          resample_f2(c, uvhat, nh);
          uvhat = nh;
        }
      }
      LevelIn L;
      L.im = lv[l];
      if (use_guide) L.guide = (ig == 0 ? cpyr : cgpyr)[l];
      if (P->method == OF_METHOD_HS) hs_base(c, P, L, uv, st);
      else if (P->method == OF_METHOD_ALT_BA) altba_base(c, P, L, uv, uvhat, P->alpha, ig != gnc - 1, st);
      else irls_base(c, P, L, uv, P->alpha, ig == 0 ? 1 : P->max_linear, st);
      HIPCHK(hipEventRecord(e1, c->stream));
      if (st && st->n_levels < OF_MAX_LEVELS) {
        st->level_h[st->n_levels] = h;
        st->level_w[st->n_levels] = w;
        st->level_stage[st->n_levels] = ig;
        st->n_levels++;
        lev_ev.push_back({e0, e1});
      }
    }
    if (gnc > 1) {  // GNC alpha schedule (classic_nl.py:180-184, ba.py:329-333)
      const double na = 1.0 - (ig + 1.0) / (gnc - 1.0);
      P->alpha = std::max(0.0, std::min(P->alpha, na));
    }
    if (c->prog_fn) {  // classic_nl.py:186-196, ba.py:132-133, alt_ba.py:175-183
      const F2 &su = P->method == OF_METHOD_ALT_BA && uvhat.p ? uvhat : uv;
      of_progress e = prog_event(c, OF_EV_STAGE_END, su.H, su.W);
      e.level = 0;
      if (c->prog_flags & OF_PROGRESS_FLOW) {
        c->prog_uv.resize(2 * (size_t)su.H * su.W);
        download_f2(c, su, c->prog_uv.data());
        e.uv = c->prog_uv.data();
      }
      HIPCHK(hipStreamSynchronize(c->stream));
      drain_solves(c);
      e.elapsed_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - c->prog_t0).count();
      c->prog_fn(c->prog_user, &e);
    }
  }
  if (P->method == OF_METHOD_BA) P->alpha = alpha_orig;  // ba.py:338-339
  if (P->method == OF_METHOD_HS && P->median_filter_size && uv.H == H && uv.W == W) {  // hs.py:94-97
    F2 t = new_f2(c, H, W);
    median2(c, uv, t, P->median_filter_size);
    uv = t;
  }
  const F2 &res = P->method == OF_METHOD_ALT_BA && uvhat.H == H ? uvhat : uv;
  if (res.H == H && res.W == W && res.p != uv_io.p)
    HIPCHK(hipMemcpyAsync(uv_io.p, res.p, sizeof(float2) * (size_t)H * uv_io.P, hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  drain_solves(c);
  if (st) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, t0, t1));
    st->preprocess_ms += ms;
    for (size_t k = 0; k < lev_ev.size(); ++k) {
      HIPCHK(hipEventElapsedTime(&ms, lev_ev[k].first, lev_ev[k].second));
      st->level_ms[k] = ms;
    }
  }
}

// estimate_flow preprocessing (interface.py:41-64): host or device RGB input
// rgb1/rgb2: (H, W, C) frames on the device, fp32 or (u8) bytes
void estimate_dev(of_ctx *c, of_params *P, const void *rgb1, const void *rgb2, bool u8, int H, int W, int C, F2 &uv,
                  of_stats *st) {
  REQUIRE(C == 1 || C == 3, OF_EINVAL, "images must be (H,W) or (H,W,3)");
  hipEvent_t t0 = timing_event(c), t1 = timing_event(c);
  HIPCHK(hipEventRecord(t0, c->stream));
  Img gray = new_img(c, H, W, 2);
  const bool guide_mode = P->guide_mode && P->method == OF_METHOD_CLASSIC_NL;
  Img guide;
  if (guide_mode) guide = new_img(c, H, W, C == 3 ? 3 : 1);
  uint32_t *mm = c->d_mm + 2 * 8;
  launch(c, "mm_init", k_mm_init, dim3(1), dim3(64), 0, mm, 1);
  const dim3 mg((unsigned)std::min<long>(((long)H * W * 3 + 255) / 256, 256));
  if (C == 3 && u8)
    launch(c, "rgb_max", k_rgb_max<uint8_t>, mg, dim3(256), 0, (const uint8_t *)rgb1, (long)H * W * 3, mm);
  else if (C == 3)
    launch(c, "rgb_max", k_rgb_max<float>, mg, dim3(256), 0, (const float *)rgb1, (long)H * W * 3, mm);
  Grid2 g = grid2(H, W);
  float *gp = guide_mode ? guide.p : (float *)nullptr;
  if (u8)
    launch(c, "rgb_prep", k_rgb_prep<uint8_t>, g.grid, g.block, 0, (const uint8_t *)rgb1, (const uint8_t *)rgb2, H, W,
           C, gray.p, gray.P, gray.ps(), gp, (const uint32_t *)mm);
  else
    launch(c, "rgb_prep", k_rgb_prep<float>, g.grid, g.block, 0, (const float *)rgb1, (const float *)rgb2, H, W, C,
           gray.p, gray.P, gray.ps(), gp, (const uint32_t *)mm);
  if (guide_mode && C == 3)
    for (int ch = 0; ch < 3; ++ch) scale_img(c, view(guide, ch, 1), 0.0f, 255.0f, 9 + ch);
  HIPCHK(hipEventRecord(t1, c->stream));
  compute_flow_dev(c, P, gray, guide, uv, st);
  if (st) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, t0, t1));
    st->preprocess_ms += ms;
  }
}

// estimate_flow on a device-resident slot, on ctx c's stream (synchronous)
void run_slot(of_ctx *c, const Slot &s, of_params *P, of_stats *st) {
  if (st) memset(st, 0, sizeof(*st));
  auto wall0 = std::chrono::steady_clock::now();
  F2 uv = new_f2(c, s.H, s.W);
  fill_f2(c, uv, 0.0f);
  estimate_dev(c, P, s.rgb1, s.rgb2, s.u8, s.H, s.W, s.C, uv, st);
  f2_to_dense(c, uv, s.uv);
  HIPCHK(hipStreamSynchronize(c->stream));
  if (st)
    st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - wall0).count();
}

int fail(of_ctx *c, const OfError &e) {
  if (c) c->err = e.msg;
  return e.code;
}

thread_local std::string g_err;

void stage_free(of_ctx *l);

}  // namespace

// Entries that compute on the context refuse while a pair stream is open on
// it: the pool's lane 0 is the context itself, and these reset its arena and
// drain its pending solves (before the try: the error path clears them too)
#define API_BEGIN(ctx)            \
  if (!ctx) return OF_EINVAL;     \
  if (ctx->pool) return fail(ctx, OfError{OF_EINVAL, "a pair stream is open on this context (of_pairs_close first)"}); \
  try {                           \
    HIPCHK(hipSetDevice(ctx->device)); \
    ctx->arena.reset();            \
    ctx->tev_used = 0;
#define API_END(ctx)                         \
  if (!ctx->pend.empty()) {                  \
    HIPCHK(hipStreamSynchronize(ctx->stream)); \
    drain_solves(ctx);                       \
  }                                          \
  flush_prof(ctx);                           \
  return OF_OK;                              \
  }                                          \
  catch (const OfError &e) {                 \
    ctx->pending.clear();                    \
    ctx->pend.clear();                       \
    ctx->ev_used = 0;                        \
    return fail(ctx, e);                     \
  }                                          \
  catch (const std::exception &e) {          \
    return fail(ctx, OfError{OF_ENOMEM, e.what()}); \
  }

// Slot copies (of_pair_upload / of_pair_download) may run while the pair
// pool computes on the context: no arena, no pending solves, and a stream of
// their own when a pool is open (the gather's)
// (the gather stream exists whenever a pool is open: of_pairs_open creates it
// with the lanes, ensure_lanes)
hipStream_t io_stream(of_ctx *c) { return c->pool ? c->gstream : c->stream; }
namespace {
void ensure_lanes(of_ctx *c, int n);
}
// a slot queued to the pair pool and not yet finished (pool_slot_busy)
bool pool_slot_busy(of_ctx *c, int slot);
#define API_BEGIN_IO(ctx)               \
  if (!ctx) return OF_EINVAL;           \
  try {                                 \
    HIPCHK(hipSetDevice(ctx->device));  \
    hipStream_t ios = io_stream(ctx);
#define API_END_IO(ctx)                                 \
  return OF_OK;                                         \
  }                                                     \
  catch (const OfError &e) {                            \
    return fail(ctx, e);                                \
  }                                                     \
  catch (const std::exception &e) {                     \
    return fail(ctx, OfError{OF_ENOMEM, e.what()});     \
  }

extern "C" {

int of_abi_version(void) { return OF_ABI_VERSION; }

int of_device_count(int *count) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  if (count) *count = n;
  return OF_OK;
}

int of_ctx_create(int device, of_ctx **out) {
  if (!out) return OF_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
    g_err = "no HIP device";
    return OF_EHIP;
  }
  of_ctx *c = new of_ctx();
  c->device = device;
  try {
    HIPCHK(hipSetDevice(device));
    create_stream(&c->stream);
    HIPCHK(hipMalloc(&c->d_state, sizeof(PcgState)));
    HIPCHK(hipHostMalloc(&c->h_state, 2 * sizeof(PcgState), hipHostMallocDefault));
    HIPCHK(hipHostMalloc(&c->h_flag, OF_SOLVE_RING * sizeof(CgFlag), hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostMalloc(&c->h_ring, OF_SOLVE_RING * sizeof(PcgState), hipHostMallocDefault));
    HIPCHK(hipHostGetDevicePointer((void **)&c->d_flag, c->h_flag, 0));
    HIPCHK(hipEventCreateWithFlags(&c->ev_state[0], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_state[1], hipEventDisableTiming));
    HIPCHK(hipMalloc(&c->d_partials, sizeof(double) * 16 * PCG_MAX_BLOCKS));
    HIPCHK(hipMalloc(&c->d_sor_sync, OF_SOR_SYNC_BYTES));
    HIPCHK(hipMalloc(&c->d_rpart, sizeof(double) * 2 * PCG_MAX_BLOCKS));
    HIPCHK(hipMalloc(&c->d_rlog, sizeof(double) * 4 * OF_SLOG_MAX));
    HIPCHK(hipFuncSetAttribute((const void *)k_sor_lex, hipFuncAttributeMaxDynamicSharedMemorySize, OF_SOR_SHM));
    HIPCHK(hipFuncSetAttribute((const void *)k_sor_pipe, hipFuncAttributeMaxDynamicSharedMemorySize, OF_SOR_PIPE_SHM));
    HIPCHK(hipFuncSetAttribute((const void *)k_sor_wg, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(OF_SORW_RING_BYTES + sizeof(SorWgShared))));
    HIPCHK(hipMalloc(&c->d_mm, sizeof(uint32_t) * 64));
    HIPCHK(hipMalloc(&c->d_norm, sizeof(double)));
    HIPCHK(hipHostMalloc(&c->h_norm, sizeof(double), hipHostMallocDefault));
  } catch (const OfError &e) {
    g_err = e.msg;
    delete c;
    return e.code;
  }
  *out = c;
  return OF_OK;
}

int of_ctx_destroy(of_ctx *c) {
  if (!c) return OF_OK;
  if (c->pool) of_pairs_close(c);
  for (of_ctx *l : c->lanes) of_ctx_destroy(l);
  c->lanes.clear();
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  stage_free(c);
  if (c->comm) ncclCommDestroy(c->comm);
  c->arena.release();
  for (auto &s : c->slots) {
    hipFree(s.rgb1);
    hipFree(s.rgb2);
    hipFree(s.uv);
  }
  if (c->own_epoch && c->epoch) hipEventDestroy(c->epoch);
  for (auto e : c->ev_pool) hipEventDestroy(e);
  for (auto e : c->tev_pool) hipEventDestroy(e);
  for (auto e : c->ev_state)
    if (e) hipEventDestroy(e);
  hipFree(c->d_state);
  hipHostFree(c->h_state);
  if (c->h_flag) hipHostFree(c->h_flag);
  if (c->h_ring) hipHostFree(c->h_ring);
  hipFree(c->d_partials);
  hipFree(c->d_sor_sync);
  if (c->d_sorp) hipFree(c->d_sorp);
  if (c->d_sor_ring) hipFree(c->d_sor_ring);
  if (c->d_gather) hipFree(c->d_gather);
  if (c->gstream) {
    hipStreamSynchronize(c->gstream);
    hipStreamDestroy(c->gstream);
  }
  hipFree(c->d_rpart);
  hipFree(c->d_rlog);
  hipFree(c->d_mm);
  hipFree(c->d_norm);
  hipHostFree(c->h_norm);
  if (c->hp) {
    hipStreamSynchronize(c->hp);
    hipStreamDestroy(c->hp);
  }
  for (auto e : c->ev_hp)
    if (e) hipEventDestroy(e);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
  return OF_OK;
}

const char *of_last_error(of_ctx *c) { return c ? c->err.c_str() : g_err.c_str(); }

int of_synchronize(of_ctx *c) {
  if (!c) return OF_EINVAL;
  return hipStreamSynchronize(c->stream) == hipSuccess ? OF_OK : OF_EHIP;
}

// Settings and profiling tables the pool's lanes read (lane 0 is the context
// itself) are refused while a pair stream is open: changing them under a
// running lane would give its pairs other arithmetic than the lanes that
// copied them at of_pairs_open, or race the lane's own writes.
#define REFUSE_WHILE_POOL(c)                                                          \
  if ((c)->pool) {                                                                   \
    (c)->err = "a pair stream is open on this context (of_pairs_close first)";       \
    return OF_EINVAL;                                                                \
  }

int of_set_option(of_ctx *c, int option, int value) {
  if (!c) return OF_EINVAL;
  REFUSE_WHILE_POOL(c)
  switch (option) {
    case OF_OPT_SOR_PIPELINE:
      c->opt_sor_pipe = value < 0 ? 0 : (value > 2 ? 2 : value);
      return OF_OK;
    case OF_OPT_FUSED_WARP:
      c->opt_fused_warp = value ? 1 : 0;
      return OF_OK;
    default:
      c->err = "unknown option";
      return OF_EINVAL;
  }
}

void pool_set_progress(PairPool *pp, of_progress_fn fn);
int of_set_progress(of_ctx *c, of_progress_fn fn, void *user, int flags) {
  if (!c) return OF_EINVAL;
  if (c->pool) pool_set_progress(c->pool, fn);  // takes effect when the pair stream closes
  else c->prog_fn = fn;
  c->prog_user = user;
  c->prog_flags = flags;
  return OF_OK;
}

int of_get_option(of_ctx *c, int option, int64_t *value) {
  if (!c || !value) return OF_EINVAL;
  switch (option) {
    case OF_OPT_SOR_PIPELINE:
      *value = c->opt_sor_pipe;
      return OF_OK;
    case OF_OPT_FUSED_WARP:
      *value = c->opt_fused_warp;
      return OF_OK;
    case OF_OPT_SOR_FALLBACKS: {
      int64_t n = c->sor_fallbacks;
      for (of_ctx *l : c->lanes) n += l->sor_fallbacks;
      *value = n;
      return OF_OK;
    }
    case OF_OPT_DEVICE_BYTES: {
      // grow-only device buffers of the context and its lanes: the arena
      // chunks, the pipelined SOR's sweep ring and the RCCL gather buffer
      auto held = [](const of_ctx *x) {
        return (int64_t)(x->arena.reserved() + x->sor_ring_cap + x->gather_cap);
      };
      int64_t n = held(c);
      for (of_ctx *l : c->lanes) n += held(l);
      *value = n;
      return OF_OK;
    }
    case OF_OPT_RCCL_NRANKS: {
      // ranks of the context's RCCL communicator as RCCL reports them (0: none)
      int n = 0;
      if (c->comm && ncclCommCount(c->comm, &n) != ncclSuccess) n = -1;
      *value = n;
      return OF_OK;
    }
    default:
      c->err = "unknown option";
      return OF_EINVAL;
  }
}

int of_set_profiling(of_ctx *c, int enable) {
  if (!c) return OF_EINVAL;
  REFUSE_WHILE_POOL(c)
  try {
    flush_prof(c);
  } catch (const OfError &e) {
    return fail(c, e);
  }
  c->prof = enable < 0 ? 0 : (enable > 3 ? 3 : enable);
  if (enable) {
    c->ktimes.clear();
    c->tl.clear();
  }
  if (c->prof == 3) {
    if (!c->epoch) {
      if (hipEventCreate(&c->epoch) != hipSuccess) return OF_EHIP;
      c->own_epoch = true;
    }
    if (hipEventRecord(c->epoch, c->stream) != hipSuccess) return OF_EHIP;
  }
  return OF_OK;
}

int of_kernel_times(of_ctx *c, int max, const char **names, double *ms, int64_t *count, double *pixels, int *n) {
  if (!c || !n) return OF_EINVAL;
  REFUSE_WHILE_POOL(c)
  int k = 0;
  for (auto &kv : c->ktimes) {
    if (k < max) {
      if (names) names[k] = kv.first.c_str();
      if (ms) ms[k] = kv.second.ms;
      if (count) count[k] = kv.second.n;
      if (pixels) pixels[k] = kv.second.px;
    }
    ++k;
  }
  *n = k;
  return OF_OK;
}

int of_kernel_timeline(of_ctx *c, int max, const char **names, double *pixels, double *t0_ms, double *t1_ms,
                       int *n) {
  if (!c || !n) return OF_EINVAL;
  REFUSE_WHILE_POOL(c)
  const int m = (int)c->tl.size();
  for (int k = 0; k < m && k < max; ++k) {
    if (names) names[k] = c->tl[k].name;
    if (pixels) pixels[k] = c->tl[k].px;
    if (t0_ms) t0_ms[k] = c->tl[k].t0;
    if (t1_ms) t1_ms[k] = c->tl[k].t1;
  }
  *n = m;
  return OF_OK;
}

int of_set_solve_log(of_ctx *c, int enable) {
  if (!c) return OF_EINVAL;
  REFUSE_WHILE_POOL(c)
  c->slog = enable ? 1 : 0;
  c->slog_rec.clear();
  return OF_OK;
}

int of_solve_log(of_ctx *c, int max, of_solve_record *out, int *n) {
  API_BEGIN(c)
  REQUIRE(n && (out || max <= 0), OF_EINVAL, "bad arguments");
  HIPCHK(hipStreamSynchronize(c->stream));
  drain_solves(c);
  const int m = (int)c->slog_rec.size();
  *n = m;
  const int k = std::min(m, max);
  if (k > 0) {
    std::vector<double> h(4 * (size_t)k);
    HIPCHK(hipMemcpy(h.data(), c->d_rlog, sizeof(double) * 4 * k, hipMemcpyDeviceToHost));
    for (int e = 0; e < k; ++e) {
      const auto &l = c->slog_rec[e];
      of_solve_record &o = out[e];
      memset(&o, 0, sizeof(o));
      o.h = l.h;
      o.w = l.w;
      o.solver = l.solver;
      o.iters = l.iters;
      o.done = l.done;
      o.true_rel = h[4 * e + 1] > 0 ? std::sqrt(h[4 * e] / h[4 * e + 1]) : 0.0;
      o.true_rel_out = h[4 * e + 3] > 0 ? std::sqrt(h[4 * e + 2] / h[4 * e + 3]) : 0.0;
      o.est_rel = l.est;
    }
  }
  API_END(c)
}

int of_solver_geometry(int H, int W, int solver, of_cg_geometry *out) {
  if (!out || solver < 0 || solver > 2) return OF_EINVAL;
  memset(out, 0, sizeof(*out));
  if (solver == OF_SOLVER_SOR) {
    if (H < 1 || W < 1) return OF_EINVAL;
    const int ns = (H + 63) / 64;
    out->grid_x = 2 * ns;
    out->grid_y = 1;
    out->rows = 64;
    out->bands = ns;
    out->blocks = 2 * ns;
    out->strip_cols = W;
    return ns <= SOR_MAXS ? OF_OK : OF_ENOTSUP;
  }
  return cg_geometry(H, W, solver == OF_SOLVER_BACKSLASH, out);
}

int of_estimate_flow(of_ctx *c, of_params *P, const float *im1, const float *im2, int H, int W, int C,
                     const float *init_uv, float *out_uv, of_stats *st) {
  API_BEGIN(c)
  REQUIRE(P && im1 && im2 && out_uv && H > 0 && W > 0, OF_EINVAL, "bad arguments");
  if (st) memset(st, 0, sizeof(*st));
  auto wall0 = std::chrono::steady_clock::now();
  const size_t n = (size_t)H * W * C;
  float *d1 = (float *)c->arena.alloc(sizeof(float) * n), *d2 = (float *)c->arena.alloc(sizeof(float) * n);
  HIPCHK(hipMemcpyAsync(d1, im1, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(d2, im2, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  F2 uv = init_uv ? upload_f2(c, init_uv, H, W) : new_f2(c, H, W);
  if (!init_uv) fill_f2(c, uv, 0.0f);
  estimate_dev(c, P, d1, d2, false, H, W, C, uv, st);
  download_f2(c, uv, out_uv);
  HIPCHK(hipStreamSynchronize(c->stream));
  if (st)
    st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - wall0).count();
  API_END(c)
}

int of_compute_flow(of_ctx *c, of_params *P, const float *images, int H, int W, int nc, const float *guide, int gc,
                    const float *init_uv, float *out_uv, of_stats *st) {
  API_BEGIN(c)
  REQUIRE(P && images && out_uv && H > 0 && W > 0 && nc >= 1, OF_EINVAL, "bad arguments");
  if (st) memset(st, 0, sizeof(*st));
  auto wall0 = std::chrono::steady_clock::now();
  Img im = new_img(c, H, W, 2 * nc);
  upload_img(c, im, images);
  Img g;
  if (guide && gc > 0) {
    g = new_img(c, H, W, gc);
    upload_img(c, g, guide);
  }
  F2 uv = init_uv ? upload_f2(c, init_uv, H, W) : new_f2(c, H, W);
  if (!init_uv) fill_f2(c, uv, 0.0f);
  compute_flow_dev(c, P, im, g, uv, st);
  download_f2(c, uv, out_uv);
  HIPCHK(hipStreamSynchronize(c->stream));
  if (st)
    st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - wall0).count();
  API_END(c)
}

int of_compute_flow_base(of_ctx *c, of_params *P, const float *images, int H, int W, int nc, const float *guide,
                         int gc, double alpha, const float *uv_in, float *out_uv) {
  API_BEGIN(c)
  REQUIRE(P && images && uv_in && out_uv, OF_EINVAL, "bad arguments");
  check_params(P);
  Img im = new_img(c, H, W, 2 * nc);
  upload_img(c, im, images);
  LevelIn L;
  L.im = im;
  if (guide && gc > 0 && P->method == OF_METHOD_CLASSIC_NL) {
    L.guide = new_img(c, H, W, gc);
    upload_img(c, L.guide, guide);
  }
  F2 uv = upload_f2(c, uv_in, H, W);
  c->prog_stage = 0;
  c->prog_level = -1;
  if (P->method == OF_METHOD_HS) hs_base(c, P, L, uv, nullptr);
  else if (P->method == OF_METHOD_ALT_BA) throw OfError{OF_ENOTSUP, "AltBA compute_flow_base needs uvhat"};
  else irls_base(c, P, L, uv, alpha, P->max_linear, nullptr);
  download_f2(c, uv, out_uv);
  HIPCHK(hipStreamSynchronize(c->stream));
  API_END(c)
}

// AltBAOpticalFlow.compute_flow_base(uv, uvhat) (alt_ba.py:189-274): one
// pyramid level of the coupled IRLS with lambda2 annealing and the Li-Osher
// median update of uvhat; returns both fields
int of_alt_ba_flow_base(of_ctx *c, of_params *P, const float *images, int H, int W, int nc, double alpha,
                        int replacement, const float *uv_in, const float *uvhat_in, float *out_uv,
                        float *out_uvhat) {
  API_BEGIN(c)
  REQUIRE(P && images && uv_in && uvhat_in && out_uv && out_uvhat && H > 0 && W > 0 && nc >= 1, OF_EINVAL,
          "bad arguments");
  REQUIRE(P->method == OF_METHOD_ALT_BA, OF_EINVAL, "of_alt_ba_flow_base needs an AltBA parameter set");
  check_params(P);
  LevelIn L;
  L.im = new_img(c, H, W, 2 * nc);
  upload_img(c, L.im, images);
  F2 uv = upload_f2(c, uv_in, H, W), uvhat = upload_f2(c, uvhat_in, H, W);
  altba_base(c, P, L, uv, uvhat, alpha, replacement != 0, nullptr);
  download_f2(c, uv, out_uv);
  download_f2(c, uvhat, out_uvhat);
  HIPCHK(hipStreamSynchronize(c->stream));
  API_END(c)
}

// ---- device-resident slots ----
int of_pair_upload(of_ctx *c, int slot, const float *im1, const float *im2, int H, int W, int C) {
  API_BEGIN_IO(c)
  REQUIRE(slot >= 0 && slot < 4096 && im1 && im2 && (C == 1 || C == 3), OF_EINVAL, "bad arguments");
  REQUIRE(!pool_slot_busy(c, slot), OF_EINVAL, "slot is queued in the pair stream (of_pairs_wait its ticket first)");
  if ((int)c->slots.size() <= slot) c->slots.resize(slot + 1);
  Slot &s = c->slots[slot];
  const size_t n = (size_t)H * W * C * sizeof(float), nu = 2 * (size_t)H * W;
  if (s.cap_rgb < n) {
    hipFree(s.rgb1);
    hipFree(s.rgb2);
    HIPCHK(hipMalloc(&s.rgb1, n));
    HIPCHK(hipMalloc(&s.rgb2, n));
    s.cap_rgb = n;
  }
  if (s.cap_uv < nu) {
    hipFree(s.uv);
    HIPCHK(hipMalloc(&s.uv, sizeof(float) * nu));
    s.cap_uv = nu;
  }
  s.H = H;
  s.W = W;
  s.C = C;
  s.u8 = false;
  HIPCHK(hipMemcpyAsync(s.rgb1, im1, n, hipMemcpyHostToDevice, ios));
  HIPCHK(hipMemcpyAsync(s.rgb2, im2, n, hipMemcpyHostToDevice, ios));
  HIPCHK(hipStreamSynchronize(ios));
  API_END_IO(c)
}

int of_pair_run(of_ctx *c, int slot, of_params *P, of_stats *st) {
  API_BEGIN(c)
  REQUIRE(slot >= 0 && slot < (int)c->slots.size() && c->slots[slot].rgb1, OF_EINVAL, "slot not uploaded");
  run_slot(c, c->slots[slot], P, st);
  API_END(c)
}

// Slots 0..nslots-1 on `lanes` concurrent pipelines.  Each lane is a child
// context (own non-blocking stream, arena, CG state and host progress flag)
// driven by its own host thread; slot s runs on lane s % lanes, so while one
// pair is in a latency-bound phase (coarse levels, solver feed, host syncs)
// another pair's kernels fill the CUs.  Every kernel is deterministic, so a
// slot's flow does not depend on the lane count.  lanes == 1 runs the slots
// in order on the ctx's own stream.
namespace {
// The batch lanes (of_pairs_run, of_pairs_run_host, the pair pool) are the
// context itself (lane 0) and its child contexts (lanes 1..), created once,
// in one consecutive batch, and kept.  The runtime binds each stream to one of
// its GPU_MAX_HW_QUEUES (4) hardware queues when the stream is created: the
// first four streams of a process get four queues, later ones share them, so
// two busy lanes can end up on one queue and serialise (43 vs 47 pairs/s).
// rocprofv3's Queue_Id per lane thread (tools/queue_map.py,
// profiles/r5_queue_map_*.txt) showed it: lanes created and destroyed per
// pool, or a fifth lane stream, collided; the context's stream plus three
// children created right after it did not.  n = child lanes wanted.
void ensure_lanes(of_ctx *c, int n) {
  const int want = std::max(n, OF_LANES_MIN - 1);
  while ((int)c->lanes.size() < want) {
    of_ctx *l = nullptr;
    const int rc = of_ctx_create(c->device, &l);
    REQUIRE(rc == OF_OK, rc, "lane context: " + g_err);
    c->lanes.push_back(l);
  }
  // the gather / slot-copy stream (of_rccl_gather_slots, io_stream) right
  // after the lanes, for every run that has lanes: N = 1 and N > 1 map their
  // streams to hardware queues the same way (one created lazily at the first
  // gather, after the copy stream, would land on a busy lane's queue)
  if (!c->gstream) create_stream(&c->gstream);
}
// profiling: the child lanes' timings into the ctx's table (lane 0, the ctx,
// records its own)
void merge_lane_prof(of_ctx *c, int lanes) {
  c->big = nullptr;
  for (int li = 1; li < lanes; ++li) {
    of_ctx *l = c->lanes[li - 1];
    for (auto &kv : l->ktimes) {
      KTime &d = c->ktimes[kv.first];
      d.ms += kv.second.ms;
      d.px += kv.second.px;
      d.n += kv.second.n;
    }
    l->ktimes.clear();
    c->tl.insert(c->tl.end(), l->tl.begin(), l->tl.end());
    l->tl.clear();
  }
}
}  // namespace

int of_pairs_run(of_ctx *c, int nslots, const of_params *P, int lanes, of_stats *st) {
  API_BEGIN(c)
  REQUIRE(P && nslots >= 1 && nslots <= (int)c->slots.size() && lanes >= 1 && lanes <= 16, OF_EINVAL,
          "bad arguments");
  for (int s = 0; s < nslots; ++s) REQUIRE(c->slots[s].rgb1 && c->slots[s].uv, OF_EINVAL, "slot not uploaded");
  REQUIRE(!c->pool, OF_EINVAL, "a pair stream is open on this context (of_pairs_close first)");
  ProgressOff quiet(c);  // batch entries never report
  lanes = std::min(lanes, nslots);
  if (lanes == 1) {
    for (int s = 0; s < nslots; ++s) {
      if (s) {
        c->arena.reset();
        c->tev_used = 0;
      }
      of_params Pc = *P;
      run_slot(c, c->slots[s], &Pc, s == 0 ? st : nullptr);
    }
  } else {
    // lane 0 is the ctx itself, lanes 1.. its long-lived children (ensure_lanes)
    ensure_lanes(c, lanes - 1);
    // big-phase token threshold in pixels.  8 1080p pairs, 2 lanes: 22.5
    // pairs/s with the token in three runs (16-18 without; 20.5 with one
    // lane) -- two lanes' fine-level CG kernels otherwise stall each other
    const double big_px = OF_BIG_PX;
    std::vector<std::thread> th;
    std::vector<OfError> errs(lanes, OfError{OF_OK, ""});
    for (int li = 0; li < lanes; ++li) {
      of_ctx *l = li ? c->lanes[li - 1] : c;
      l->prof = c->prof;
      l->opt_sor_pipe = c->opt_sor_pipe;
      l->opt_fused_warp = c->opt_fused_warp;
      if (l != c) l->epoch = c->epoch;
      l->big = big_px > 0 ? &c->big_own : nullptr;
      l->big_px = big_px;
      th.emplace_back([c, l, li, lanes, nslots, P, st, &errs] {
        try {
          HIPCHK(hipSetDevice(l->device));
          for (int s = li; s < nslots; s += lanes) {
            l->arena.reset();
            l->tev_used = 0;
            of_params Pc = *P;
            run_slot(l, c->slots[s], &Pc, s == 0 ? st : nullptr);
          }
          if (l != c) flush_prof(l);
        } catch (const OfError &e) {
          errs[li] = e;
          hipStreamSynchronize(l->stream);
          l->pending.clear();
          l->ev_used = 0;
        } catch (const std::exception &e) {
          errs[li] = OfError{OF_ENOMEM, e.what()};
        }
      });
    }
    for (auto &t : th) t.join();
    merge_lane_prof(c, lanes);
    for (auto &e : errs)
      if (e.code != OF_OK) throw e;
  }
  API_END(c)
}

namespace {
void stage_alloc(of_ctx *l, of_ctx *parent, size_t in_bytes, size_t out_floats) {
  if (!l->hs) {
    l->hs = new HostStage();
    if (l == parent) {
      create_stream(&l->hs->copy);
      l->hs->own_copy = true;
    }
    for (int b = 0; b < 2; ++b) {
      HIPCHK(hipEventCreateWithFlags(&l->hs->ev_in[b], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&l->hs->ev_conv[b], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&l->hs->ev_out[b], hipEventDisableTiming));
    }
  }
  HostStage &h = *l->hs;
  if (!h.own_copy) h.copy = parent->hs->copy;
  if (h.cap_in < in_bytes) {
    for (int b = 0; b < 2; ++b) {
      HIPCHK(hipEventSynchronize(h.ev_in[b]));
      HIPCHK(hipEventSynchronize(h.ev_conv[b]));
      if (h.pin_in[b]) hipHostFree(h.pin_in[b]);
      hipFree(h.d_in[b]);
      HIPCHK(hipHostMalloc((void **)&h.pin_in[b], in_bytes, hipHostMallocDefault));
      HIPCHK(hipMalloc((void **)&h.d_in[b], in_bytes));
    }
    h.cap_in = in_bytes;
  }
  if (h.cap_out < out_floats) {
    for (int b = 0; b < 2; ++b) {
      HIPCHK(hipEventSynchronize(h.ev_out[b]));
      if (h.pin_out[b]) hipHostFree(h.pin_out[b]);
      HIPCHK(hipHostMalloc((void **)&h.pin_out[b], sizeof(float) * out_floats, hipHostMallocDefault));
    }
    h.cap_out = out_floats;
  }
}

void stage_free(of_ctx *l) {
  if (!l->hs) return;
  HostStage &h = *l->hs;
  for (int b = 0; b < 2; ++b)
    for (hipEvent_t e : {h.ev_in[b], h.ev_out[b]})
      if (e) hipEventSynchronize(e);
  for (int b = 0; b < 2; ++b) {
    if (h.pin_in[b]) hipHostFree(h.pin_in[b]);
    if (h.pin_out[b]) hipHostFree(h.pin_out[b]);
    hipFree(h.d_in[b]);
    for (hipEvent_t e : {h.ev_in[b], h.ev_conv[b], h.ev_out[b]})
      if (e) hipEventDestroy(e);
  }
  if (h.own_copy && h.copy) {
    hipStreamSynchronize(h.copy);
    hipStreamDestroy(h.copy);
  }
  delete l->hs;
  l->hs = nullptr;
}

// One lane's share of of_pairs_run_host: pairs k = first, first + step, ...
// Per pair j (buffer b = j & 1): host bytes -> pinned -> device on the copy
// stream (issued while pair j-1 computes), estimate_flow on the lane stream
// straight from the bytes, flow -> slot k's device buffer (kept for the RCCL
// gather) -> pinned on the copy stream -> caller's buffer (while pair j+1
// computes).
void run_host_lane(of_ctx *c, of_ctx *l, int first, int step, int npairs, const uint8_t *const *im1,
                   const uint8_t *const *im2, int H, int W, int C, const of_params *P, float *const *out_uv,
                   of_stats *st) {
  HostStage &h = *l->hs;
  const size_t nb = (size_t)H * W * C, nu = 2 * (size_t)H * W;
  std::vector<int> ks;
  for (int k = first; k < npairs; k += step) ks.push_back(k);
  auto prefetch = [&](int j) {
    const int b = j & 1, k = ks[j];
    HIPCHK(hipEventSynchronize(h.ev_in[b]));  // pinned buffer b free (its last H2D done)
    memcpy(h.pin_in[b], im1[k], nb);
    memcpy(h.pin_in[b] + nb, im2[k], nb);
    HIPCHK(hipEventSynchronize(h.ev_conv[b]));  // device buffer b no longer read (pair j-2 done)
    HIPCHK(hipMemcpyAsync(h.d_in[b], h.pin_in[b], 2 * nb, hipMemcpyHostToDevice, h.copy));
    HIPCHK(hipEventRecord(h.ev_in[b], h.copy));
  };
  // pair j's flow: wait for its kernels on the host, then D2H on the shared
  // copy stream into pinned buffer b and out to the caller
  auto finish = [&](int j) {
    const int b = j & 1;
    HIPCHK(hipEventSynchronize(h.ev_conv[b]));
    HIPCHK(hipMemcpyAsync(h.pin_out[b], c->slots[ks[j]].uv, sizeof(float) * nu, hipMemcpyDeviceToHost, h.copy));
    HIPCHK(hipEventRecord(h.ev_out[b], h.copy));
    HIPCHK(hipEventSynchronize(h.ev_out[b]));
    memcpy(out_uv[ks[j]], h.pin_out[b], sizeof(float) * nu);
  };
  // the host copies of pair j+1 (in) and pair j-1 (out) run on a helper
  // thread while this thread drives pair j's kernels
  std::thread io;
  OfError io_err{OF_OK, ""};
  auto join_io = [&] {
    if (io.joinable()) io.join();
    if (io_err.code != OF_OK) throw io_err;
  };
  if (!ks.empty()) prefetch(0);
  for (int j = 0; j < (int)ks.size(); ++j) {
    const int b = j & 1, k = ks[j];
    join_io();
    l->arena.reset();
    l->tev_used = 0;
    HIPCHK(hipStreamWaitEvent(l->stream, h.ev_in[b], 0));
    Slot s;
    s.rgb1 = h.d_in[b];
    s.rgb2 = h.d_in[b] + nb;
    s.u8 = true;
    s.uv = c->slots[k].uv;
    s.H = H;
    s.W = W;
    s.C = C;
    io = std::thread([&, j] {
      try {
        HIPCHK(hipSetDevice(l->device));
        if (j + 1 < (int)ks.size()) prefetch(j + 1);
        if (j) finish(j - 1);
      } catch (const OfError &e) {
        io_err = e;
      }
    });
    try {
      of_params Pc = *P;
      run_slot(l, s, &Pc, k == 0 ? st : nullptr);
    } catch (...) {
      if (io.joinable()) io.join();
      throw;
    }
    HIPCHK(hipEventRecord(h.ev_conv[b], l->stream));  // frames of buffer b consumed, flow k complete
  }
  join_io();
  if (!ks.empty()) finish((int)ks.size() - 1);
}
}  // namespace

// Host-to-host batch (SURVEY.md §8d headline: wall clock including the H2D of
// the uint8 pair and the D2H of uv): pairs are read from caller-owned (H, W, C)
// uint8 frames and the flows written to caller-owned planar 2 x H x W fp32
// buffers, `lanes` pairs in flight as in of_pairs_run.  Slots 0..npairs-1 keep
// each pair's flow on the device afterwards (of_rccl_gather_flows,
// of_pair_download).
int of_pairs_run_host(of_ctx *c, int npairs, const uint8_t *const *im1, const uint8_t *const *im2, int H, int W,
                      int C, const of_params *P, int lanes, float *const *out_uv, of_stats *st) {
  API_BEGIN(c)
  REQUIRE(P && im1 && im2 && out_uv && npairs >= 1 && npairs <= 4096 && H > 0 && W > 0 && (C == 1 || C == 3) &&
              lanes >= 1 && lanes <= 16,
          OF_EINVAL, "bad arguments");
  for (int k = 0; k < npairs; ++k) REQUIRE(im1[k] && im2[k] && out_uv[k], OF_EINVAL, "null pair buffer");
  REQUIRE(!c->pool, OF_EINVAL, "a pair stream is open on this context (of_pairs_close first)");
  ProgressOff quiet(c);  // batch entries never report
  if ((int)c->slots.size() < npairs) c->slots.resize(npairs);
  const size_t nu = 2 * (size_t)H * W;
  for (int k = 0; k < npairs; ++k) {
    Slot &s = c->slots[k];
    if (s.cap_uv < nu) {
      hipFree(s.uv);
      HIPCHK(hipMalloc(&s.uv, sizeof(float) * nu));
      s.cap_uv = nu;
    }
    // the slot now holds this batch's flow; frames of an earlier
    // of_pair_upload (possibly of another size) are dropped so that
    // of_pair_run / of_pairs_run refuse the slot until it is re-uploaded
    if (s.rgb1 || s.rgb2) {
      HIPCHK(hipStreamSynchronize(c->stream));
      hipFree(s.rgb1);
      hipFree(s.rgb2);
      s.rgb1 = s.rgb2 = nullptr;
      s.cap_rgb = 0;
    }
    s.H = H;
    s.W = W;
    s.C = C;
  }
  lanes = std::min(lanes, npairs);
  if (lanes > 1) ensure_lanes(c, lanes - 1);  // lane streams before the copy stream (ensure_lanes)
  for (int li = 0; li < lanes; ++li) stage_alloc(li ? c->lanes[li - 1] : c, c, 2 * (size_t)H * W * C, nu);
  if (lanes == 1) {
    run_host_lane(c, c, 0, 1, npairs, im1, im2, H, W, C, P, out_uv, st);
  } else {
    std::vector<std::thread> th;
    std::vector<OfError> errs(lanes, OfError{OF_OK, ""});
    for (int li = 0; li < lanes; ++li) {
      of_ctx *l = li ? c->lanes[li - 1] : c;
      l->prof = c->prof;
      l->opt_sor_pipe = c->opt_sor_pipe;
      l->opt_fused_warp = c->opt_fused_warp;
      if (l != c) l->epoch = c->epoch;
      l->big = OF_BIG_PX > 0 ? &c->big_own : nullptr;
      l->big_px = OF_BIG_PX;
      th.emplace_back([=, &errs] {
        try {
          HIPCHK(hipSetDevice(l->device));
          run_host_lane(c, l, li, lanes, npairs, im1, im2, H, W, C, P, out_uv, st);
          if (l != c) flush_prof(l);
        } catch (const OfError &e) {
          errs[li] = e;
          hipStreamSynchronize(l->stream);
          if (l->hs) hipStreamSynchronize(l->hs->copy);
          l->pending.clear();
          l->ev_used = 0;
        } catch (const std::exception &e) {
          errs[li] = OfError{OF_ENOMEM, e.what()};
        }
      });
    }
    for (auto &t : th) t.join();
    merge_lane_prof(c, lanes);
    for (auto &e : errs)
      if (e.code != OF_OK) throw e;
  }
  API_END(c)
}

// ---- streaming batch: a persistent pool of lanes fed from a queue --------
namespace {
struct PairJob {
  const uint8_t *im1, *im2;  // host frames (of_pairs_submit) ...
  float *out;
  int64_t ticket;
  Slot dev;                  // ... or a device-resident slot (of_pairs_submit_slots)
  bool on_dev = false;
  int slot = -1;             // that slot's index
};
}  // namespace

struct PairPool {
  int H = 0, W = 0, C = 0;
  of_params P;
  std::vector<of_ctx *> lanes;  // the ctx and its lane children (of_pairs_run's lanes), not owned
  of_progress_fn prog_fn = nullptr;  // the ctx's progress callback, off while the pool runs
  std::vector<float *> d_uv;  // 2 device flow buffers per lane
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv_job, cv_done;
  std::deque<PairJob> q;
  bool closing = false;
  int64_t next_ticket = 0;
  std::vector<uint8_t> done;  // by ticket
  std::map<int, int> busy;    // device slot -> its queued or running jobs (of_pairs_submit_slots)
  OfError err{OF_OK, ""};
};

extern "C++" bool pool_slot_busy(of_ctx *c, int slot) {
  PairPool *pp = c->pool;
  if (!pp) return false;
  std::lock_guard<std::mutex> lk(pp->m);
  auto it = pp->busy.find(slot);
  return it != pp->busy.end() && it->second > 0;
}

void pool_set_progress(PairPool *pp, of_progress_fn fn) { pp->prog_fn = fn; }

namespace {
// One lane of the pool: the per-pair pipeline of run_host_lane (pinned and
// device double buffers, H2D of the next pair and D2H of the previous one on
// a helper thread while this thread drives a pair's kernels), but pairs come
// from the pool's queue as they are submitted, so a lane never drains between
// the caller's chunks.  A pair's flow is written out as soon as no next pair
// is waiting, so of_pairs_wait never waits for a later submission.
void pool_lane(of_ctx *c, PairPool *pp, int li) {
  of_ctx *l = pp->lanes[li];
  HostStage &h = *l->hs;
  const int H = pp->H, W = pp->W, C = pp->C;
  const size_t nb = (size_t)H * W * C, nu = 2 * (size_t)H * W;
  float *duv[2] = {pp->d_uv[2 * li], pp->d_uv[2 * li + 1]};
  auto pop = [&](PairJob &j, const bool *stop) {
    std::unique_lock<std::mutex> lk(pp->m);
    pp->cv_job.wait(lk, [&] { return !pp->q.empty() || pp->closing || (stop && *stop); });
    if (pp->q.empty()) return false;
    j = pp->q.front();
    pp->q.pop_front();
    return true;
  };
  auto prefetch = [&](int b, const PairJob &j) {
    if (j.on_dev) return;  // frames already in HBM
    HIPCHK(hipEventSynchronize(h.ev_in[b]));
    memcpy(h.pin_in[b], j.im1, nb);
    memcpy(h.pin_in[b] + nb, j.im2, nb);
    HIPCHK(hipEventSynchronize(h.ev_conv[b]));
    HIPCHK(hipMemcpyAsync(h.d_in[b], h.pin_in[b], 2 * nb, hipMemcpyHostToDevice, h.copy));
    HIPCHK(hipEventRecord(h.ev_in[b], h.copy));
  };
  auto finish = [&](int b, const PairJob &j) {
    HIPCHK(hipEventSynchronize(h.ev_conv[b]));
    if (!j.on_dev) {  // a device slot's flow stays in its slot
      HIPCHK(hipMemcpyAsync(h.pin_out[b], duv[b], sizeof(float) * nu, hipMemcpyDeviceToHost, h.copy));
      HIPCHK(hipEventRecord(h.ev_out[b], h.copy));
      HIPCHK(hipEventSynchronize(h.ev_out[b]));
      memcpy(j.out, h.pin_out[b], sizeof(float) * nu);
    }
    {
      std::lock_guard<std::mutex> lk(pp->m);
      if (j.on_dev) --pp->busy[j.slot];
      pp->done[j.ticket] = 1;
    }
    pp->cv_done.notify_all();
  };
  PairJob jobs[2];
  if (!pop(jobs[0], nullptr)) return;
  prefetch(0, jobs[0]);
  int b = 0, pending = -1;  // pending: buffer of a computed pair not yet written out
  for (;;) {
    l->arena.reset();
    l->tev_used = 0;
    Slot s;
    if (jobs[b].on_dev) {
      s = jobs[b].dev;
    } else {
      HIPCHK(hipStreamWaitEvent(l->stream, h.ev_in[b], 0));
      s.rgb1 = h.d_in[b];
      s.rgb2 = h.d_in[b] + nb;
      s.u8 = true;
      s.uv = duv[b];
      s.H = H;
      s.W = W;
      s.C = C;
    }
    bool computed = false, got = false;
    OfError io_err{OF_OK, ""};
    std::thread io([&, b, pending] {
      try {
        HIPCHK(hipSetDevice(l->device));
        if (pending >= 0) finish(pending, jobs[pending]);
        got = pop(jobs[b ^ 1], &computed);
        if (got) prefetch(b ^ 1, jobs[b ^ 1]);
      } catch (const OfError &e) {
        io_err = e;
      }
    });
    auto release_io = [&] {
      {
        std::lock_guard<std::mutex> lk(pp->m);
        computed = true;
      }
      pp->cv_job.notify_all();
      io.join();
    };
    try {
      of_params Pc = pp->P;
      run_slot(l, s, &Pc, nullptr);
      HIPCHK(hipEventRecord(h.ev_conv[b], l->stream));
    } catch (...) {
      release_io();
      throw;
    }
    release_io();
    if (io_err.code != OF_OK) throw io_err;
    pending = b;
    if (!got) {
      finish(b, jobs[b]);
      pending = -1;
      if (!pop(jobs[b ^ 1], nullptr)) return;
      prefetch(b ^ 1, jobs[b ^ 1]);
    }
    b ^= 1;
  }
}
}  // namespace

// Streaming batch (host I/O overlapped with the GPU):
// of_pairs_open starts `lanes` pipelines (child contexts, one host thread
// each) that take (H, W, C) uint8 pairs from a queue; of_pairs_submit queues
// pairs and returns at once; of_pairs_wait blocks until a pair's flow is in
// the caller's buffer.  Flows equal of_pairs_run_host's with the same lanes
// (bitwise): lanes == 1 keeps estimate_flow's geometry, lanes >= 2 share the
// fine-solve token (two pairs' fine CG solves side by side).
int of_pairs_open(of_ctx *c, int H, int W, int C, const of_params *P, int lanes) {
  API_BEGIN(c)
  REQUIRE(!c->pool, OF_EINVAL, "a pair stream is already open on this context");
  REQUIRE(P && H > 0 && W > 0 && (C == 1 || C == 3) && lanes >= 1 && lanes <= 16, OF_EINVAL, "bad arguments");
  check_params(P);
  std::unique_ptr<PairPool> pp(new PairPool());
  pp->H = H;
  pp->W = W;
  pp->C = C;
  pp->P = *P;
  const size_t nu = 2 * (size_t)H * W;
  ensure_lanes(c, lanes - 1);  // lane streams before the copy stream (ensure_lanes)
  try {
    // the pool runs on the context's long-lived lane children (the ones
    // of_pairs_run / of_pairs_run_host use): lanes created and destroyed per
    // pool would shift the runtime's stream -> hardware-queue mapping for
    // the lanes created after them (create_stream)
    for (int li = 0; li < lanes; ++li) {
      of_ctx *l = li ? c->lanes[li - 1] : c;
      pp->lanes.push_back(l);
      if (l != c) l->prof = 0;
      l->opt_sor_pipe = c->opt_sor_pipe;
      l->opt_fused_warp = c->opt_fused_warp;
      l->big = lanes > 1 && OF_BIG_PX > 0 ? &c->big_own : nullptr;
      l->big_px = OF_BIG_PX;
      stage_alloc(l, c, 2 * (size_t)H * W * C, nu);
      for (int b = 0; b < 2; ++b) {
        float *d = nullptr;
        HIPCHK(hipMalloc(&d, sizeof(float) * nu));
        pp->d_uv.push_back(d);
      }
    }
  } catch (...) {
    for (float *d : pp->d_uv) hipFree(d);
    throw;
  }
  PairPool *raw = pp.release();
  c->pool = raw;
  raw->prog_fn = c->prog_fn;  // lane 0 is the ctx: batch lanes never report
  c->prog_fn = nullptr;
  for (int li = 0; li < lanes; ++li)
    raw->th.emplace_back([c, raw, li] {
      try {
        HIPCHK(hipSetDevice(raw->lanes[li]->device));
        pool_lane(c, raw, li);
      } catch (const OfError &e) {
        std::lock_guard<std::mutex> lk(raw->m);
        if (raw->err.code == OF_OK) raw->err = e;
        raw->closing = true;
      } catch (const std::exception &e) {
        std::lock_guard<std::mutex> lk(raw->m);
        if (raw->err.code == OF_OK) raw->err = OfError{OF_ENOMEM, e.what()};
        raw->closing = true;
      }
      raw->cv_done.notify_all();
      raw->cv_job.notify_all();
    });
  API_END(c)
}

// queue n pairs (caller-owned (H, W, C) uint8 frames and planar 2 x H x W fp32
// outputs, all kept alive until waited for); tickets first .. first + n - 1
int of_pairs_submit(of_ctx *c, int n, const uint8_t *const *im1, const uint8_t *const *im2, float *const *out_uv,
                    int64_t *first_ticket) {
  if (!c) return OF_EINVAL;
  PairPool *pp = c->pool;
  if (!pp || n < 1 || !im1 || !im2 || !out_uv) {
    c->err = pp ? "bad arguments" : "no pair stream open (of_pairs_open)";
    return OF_EINVAL;
  }
  for (int k = 0; k < n; ++k)
    if (!im1[k] || !im2[k] || !out_uv[k]) {
      c->err = "null pair buffer";
      return OF_EINVAL;
    }
  {
    std::lock_guard<std::mutex> lk(pp->m);
    if (pp->err.code != OF_OK) {
      c->err = pp->err.msg;
      return pp->err.code;
    }
    if (pp->closing) {
      c->err = "pair stream closing";
      return OF_EINVAL;
    }
    if (first_ticket) *first_ticket = pp->next_ticket;
    for (int k = 0; k < n; ++k) {
      PairJob j;
      j.im1 = im1[k];
      j.im2 = im2[k];
      j.out = out_uv[k];
      j.ticket = pp->next_ticket++;
      pp->q.push_back(j);
      pp->done.push_back(0);
    }
  }
  pp->cv_job.notify_all();
  return OF_OK;
}

// queue n device-resident pairs (slots of this context, of_pair_upload); each
// flow stays in its slot.  A slot is read and written by the lane that takes
// it, so it must not be submitted again (or re-uploaded) before its ticket is
// waited for.
int of_pairs_submit_slots(of_ctx *c, int n, const int *slots, int64_t *first_ticket) {
  if (!c) return OF_EINVAL;
  PairPool *pp = c->pool;
  if (!pp || n < 1 || !slots) {
    c->err = pp ? "bad arguments" : "no pair stream open (of_pairs_open)";
    return OF_EINVAL;
  }
  for (int k = 0; k < n; ++k) {
    const int sl = slots[k];
    if (sl < 0 || sl >= (int)c->slots.size() || !c->slots[sl].rgb1 || !c->slots[sl].uv) {
      c->err = "slot not uploaded";
      return OF_EINVAL;
    }
    if (c->slots[sl].H != pp->H || c->slots[sl].W != pp->W) {
      c->err = "slot frame size differs from the stream's";
      return OF_EINVAL;
    }
  }
  {
    std::lock_guard<std::mutex> lk(pp->m);
    if (pp->err.code != OF_OK) {
      c->err = pp->err.msg;
      return pp->err.code;
    }
    if (pp->closing) {
      c->err = "pair stream closing";
      return OF_EINVAL;
    }
    for (int k = 0; k < n; ++k) {
      auto it = pp->busy.find(slots[k]);
      int dup = 0;
      for (int q = 0; q < k; ++q) dup += slots[q] == slots[k];
      if ((it != pp->busy.end() && it->second > 0) || dup) {
        c->err = "slot already queued in the pair stream (of_pairs_wait its ticket first)";
        return OF_EINVAL;
      }
    }
    if (first_ticket) *first_ticket = pp->next_ticket;
    for (int k = 0; k < n; ++k) {
      PairJob j;
      j.im1 = j.im2 = nullptr;
      j.out = nullptr;
      j.ticket = pp->next_ticket++;
      j.dev = c->slots[slots[k]];
      j.on_dev = true;
      j.slot = slots[k];
      ++pp->busy[slots[k]];
      pp->q.push_back(j);
      pp->done.push_back(0);
    }
  }
  pp->cv_job.notify_all();
  return OF_OK;
}

// block until pair `ticket`'s flow has been written (a lane's error is
// returned here, and by every later call)
int of_pairs_wait(of_ctx *c, int64_t ticket) {
  if (!c) return OF_EINVAL;
  PairPool *pp = c->pool;
  if (!pp) {
    c->err = "no pair stream open (of_pairs_open)";
    return OF_EINVAL;
  }
  std::unique_lock<std::mutex> lk(pp->m);
  if (ticket < 0 || ticket >= pp->next_ticket) {
    c->err = "unknown ticket";
    return OF_EINVAL;
  }
  pp->cv_done.wait(lk, [&] { return pp->done[ticket] || pp->err.code != OF_OK; });
  if (!pp->done[ticket]) {
    c->err = pp->err.msg;
    return pp->err.code;
  }
  return OF_OK;
}

// finish every queued pair, stop the lanes and release them
int of_pairs_close(of_ctx *c) {
  if (!c) return OF_EINVAL;
  PairPool *pp = c->pool;
  if (!pp) return OF_OK;
  {
    std::lock_guard<std::mutex> lk(pp->m);
    pp->closing = true;
  }
  pp->cv_job.notify_all();
  for (auto &t : pp->th) t.join();
  for (of_ctx *l : pp->lanes) {  // the lanes stay with the context
    l->big = nullptr;
    l->arena.reset();
  }
  c->prog_fn = pp->prog_fn;
  hipSetDevice(c->device);
  for (float *d : pp->d_uv) hipFree(d);
  const OfError e = pp->err;
  delete pp;
  c->pool = nullptr;
  if (e.code != OF_OK) {
    c->err = e.msg;
    return e.code;
  }
  return OF_OK;
}

int of_pair_download(of_ctx *c, int slot, float *out_uv) {
  API_BEGIN_IO(c)
  REQUIRE(slot >= 0 && slot < (int)c->slots.size() && c->slots[slot].uv && out_uv, OF_EINVAL, "bad slot");
  REQUIRE(!pool_slot_busy(c, slot), OF_EINVAL, "slot is queued in the pair stream (of_pairs_wait its ticket first)");
  Slot &s = c->slots[slot];
  HIPCHK(hipMemcpyAsync(out_uv, s.uv, sizeof(float) * 2 * (size_t)s.H * s.W, hipMemcpyDeviceToHost, ios));
  HIPCHK(hipStreamSynchronize(ios));
  API_END_IO(c)
}

// ---- RCCL gather: one process per GPU ----
int of_rccl_unique_id(char *out128) {
  if (!out128) return OF_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return OF_ERCCL;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  memcpy(out128, &id, 128);
  return OF_OK;
}

int of_rccl_init(of_ctx *c, const char *id128, int nranks, int rank) {
  API_BEGIN(c)
  REQUIRE(id128 && nranks >= 1 && rank >= 0 && rank < nranks, OF_EINVAL, "bad arguments");
  ncclUniqueId id;
  memcpy(&id, id128, 128);
  ensure_lanes(c, 0);  // the lanes and the gather stream, in the order a pool would create them
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
  REQUIRE(r == ncclSuccess, OF_ERCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  c->nranks = nranks;
  c->rank = rank;
  API_END(c)
}

int of_rccl_gather_flows(of_ctx *c, int nslots, float *out_uv_rank0) {
  return of_rccl_gather_slots(c, 0, nslots, out_uv_rank0);
}

// May run while a pair stream is open on this context, whose lane 0 is the
// context itself (bench.py gathers step s's slots while step s + 1 computes):
// so no API_BEGIN / API_END here -- they reset the context's arena and drain
// its pending solves under the lane thread -- and the gather's copies and
// RCCL calls go to a stream of its own (the slots' flows are complete: a
// ticket is done only after its lane's stream reached the end of the pair).
int of_rccl_gather_slots(of_ctx *c, int first, int nslots, float *out_uv_rank0) {
  if (!c) return OF_EINVAL;
  try {
  HIPCHK(hipSetDevice(c->device));
  REQUIRE(c->comm, OF_EINVAL, "of_rccl_init first");
  if (!c->gstream) ensure_lanes(c, 0);  // (never while a pool is open: of_pairs_open made it)
  REQUIRE(first >= 0 && nslots >= 1 && first + nslots <= (int)c->slots.size(), OF_EINVAL, "bad slot range");
  Slot *sl = c->slots.data() + first;
  const int H = sl[0].H, W = sl[0].W;
  for (int s = 0; s < nslots; ++s)
    REQUIRE(sl[s].uv && sl[s].H == H && sl[s].W == W, OF_EINVAL, "slots must share one size");
  const size_t per = 2 * (size_t)H * W;
  float *recv = nullptr;
  if (c->rank == 0) {  // one grow-only receive buffer per context (the call ends in a sync)
    const size_t need = sizeof(float) * per * nslots * c->nranks;
    if (need > c->gather_cap) {
      if (c->d_gather) HIPCHK(hipFree(c->d_gather));
      c->d_gather = nullptr;
      c->gather_cap = 0;
      HIPCHK(hipMalloc(&c->d_gather, need));
      c->gather_cap = need;
    }
    recv = c->d_gather;
  }
  // rank 0's own slots first: nothing that can throw runs between
  // ncclGroupStart and ncclGroupEnd, so a failed copy cannot leave a group open
  if (c->rank == 0)
    for (int s = 0; s < nslots; ++s)
      HIPCHK(hipMemcpyAsync(recv + per * s, sl[s].uv, sizeof(float) * per, hipMemcpyDeviceToDevice, c->gstream));
  ncclResult_t r = ncclGroupStart();
  for (int s = 0; s < nslots && r == ncclSuccess; ++s) {
    if (c->rank == 0) {
      for (int src = 1; src < c->nranks && r == ncclSuccess; ++src)
        r = ncclRecv(recv + per * ((size_t)src * nslots + s), per, ncclFloat, src, c->comm, c->gstream);
    } else {
      r = ncclSend(sl[s].uv, per, ncclFloat, 0, c->comm, c->gstream);
    }
  }
  ncclResult_t r2 = ncclGroupEnd();
  REQUIRE(r == ncclSuccess && r2 == ncclSuccess, OF_ERCCL,
          std::string("rccl gather: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
  if (c->rank == 0 && out_uv_rank0)
    HIPCHK(hipMemcpyAsync(out_uv_rank0, recv, sizeof(float) * per * nslots * c->nranks, hipMemcpyDeviceToHost,
                          c->gstream));
  HIPCHK(hipStreamSynchronize(c->gstream));
  return OF_OK;
  } catch (const OfError &e) {
    return fail(c, e);
  } catch (const std::exception &e) {
    return fail(c, OfError{OF_ENOMEM, e.what()});
  }
}

int of_rccl_finalize(of_ctx *c) {
  if (!c) return OF_EINVAL;
  if (c->comm) ncclCommDestroy(c->comm);
  c->comm = nullptr;
  return OF_OK;
}

// ---- stage entries ----
int of_preprocess(of_ctx *c, const float *rgb1, const float *rgb2, int H, int W, float *gray_pair, float *lab) {
  API_BEGIN(c)
  REQUIRE(rgb1 && rgb2 && gray_pair, OF_EINVAL, "bad arguments");
  const size_t n = (size_t)H * W * 3;
  float *d1 = (float *)c->arena.alloc(sizeof(float) * n), *d2 = (float *)c->arena.alloc(sizeof(float) * n);
  HIPCHK(hipMemcpyAsync(d1, rgb1, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(d2, rgb2, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  Img gray = new_img(c, H, W, 2), g3 = new_img(c, H, W, 3);
  uint32_t *mm = c->d_mm + 2 * 8;
  launch(c, "mm_init", k_mm_init, dim3(1), dim3(64), 0, mm, 1);
  launch(c, "rgb_max", k_rgb_max<float>, dim3((unsigned)std::min<size_t>((n + 255) / 256, 256)), dim3(256), 0,
         (const float *)d1, (long)n, mm);
  Grid2 g = grid2(H, W);
  launch(c, "rgb_prep", k_rgb_prep<float>, g.grid, g.block, 0, (const float *)d1, (const float *)d2, H, W, 3, gray.p, gray.P,
         gray.ps(), g3.p, (const uint32_t *)mm);
  for (int ch = 0; ch < 3; ++ch) scale_img(c, view(g3, ch, 1), 0.0f, 255.0f, 9 + ch);
  download_img(c, gray, gray_pair);
  if (lab) download_img(c, g3, lab);
  HIPCHK(hipStreamSynchronize(c->stream));
  API_END(c)
}

int of_rof_texture(of_ctx *c, const float *im, int H, int W, int C, double theta, int iters, double alp, float *out) {
  API_BEGIN(c)
  REQUIRE(im && out && C >= 1, OF_EINVAL, "bad arguments");
  Img m = new_img(c, H, W, C);
  upload_img(c, m, im);
  Img t = rof_texture(c, m, theta, iters, alp);
  download_img(c, t, out);
  HIPCHK(hipStreamSynchronize(c->stream));
  API_END(c)
}

int of_pyramid_level(of_ctx *c, const float *im, int H, int W, int C, const double *kern, int ksize, double ratio,
                     float *out, int *outH, int *outW) {
  API_BEGIN(c)
  REQUIRE(im && out && kern && ksize >= 1 && ksize <= 5 && (ksize & 1), OF_EINVAL, "bad arguments");
  Img m = new_img(c, H, W, C);
  upload_img(c, m, im);
  Img o = pyramid_step(c, m, make_taps(kern, ksize, ksize), ratio);
  download_img(c, o, out);
  if (outH) *outH = o.H;
  if (outW) *outW = o.W;
  HIPCHK(hipStreamSynchronize(c->stream));
  API_END(c)
}

int of_resample_flow(of_ctx *c, const float *uv, int H, int W, int nH, int nW, float *out) {
  API_BEGIN(c)
  REQUIRE(uv && out, OF_EINVAL, "bad arguments");
  F2 a = upload_f2(c, uv, H, W);
  if (H == nH && W == nW) {
    download_f2(c, a, out);
  } else {
    F2 b = new_f2(c, nH, nW);
    resample_f2(c, a, b);
    download_f2(c, b, out);
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  API_END(c)
}

int of_partial_deriv(of_ctx *c, const float *images, int H, int W, int nc, const float *uv, int interp,
                     const double *filt, double blend, float *It, float *Ix, float *Iy) {
  API_BEGIN(c)
  REQUIRE(images && uv && filt && It && Ix && Iy && nc >= 1 && nc <= OF_MAX_NC, OF_EINVAL, "bad arguments");
  REQUIRE(interp >= 0 && interp <= 2, OF_EINVAL, "Unknown interpolation method");
  Img im = new_img(c, H, W, 2 * nc);
  upload_img(c, im, images);
  F2 f = upload_f2(c, uv, H, W);
  LevelDeriv D = level_deriv(c, im, nc, interp, filt, blend);
  Img a = new_img(c, H, W, nc), b = new_img(c, H, W, nc), d = new_img(c, H, W, nc);
  partial_deriv(c, D, interp, f, a, b, d);
  download_img(c, a, It);
  download_img(c, b, Ix);
  download_img(c, d, Iy);
  HIPCHK(hipStreamSynchronize(c->stream));
  API_END(c)
}

int of_flow_operator(of_ctx *c, const of_params *P, double alpha, const float *uv, const float *duv, const float *It,
                     const float *Ix, const float *Iy, int H, int W, int nc, float *coef, float *rhs) {
  API_BEGIN(c)
  REQUIRE(P && uv && It && Ix && Iy && coef && rhs && nc >= 1, OF_EINVAL, "bad arguments");
  F2 f = upload_f2(c, uv, H, W);
  F2 df;
  if (duv) df = upload_f2(c, duv, H, W);
  Img a = new_img(c, H, W, nc), b = new_img(c, H, W, nc), d = new_img(c, H, W, nc);
  upload_img(c, a, It);
  upload_img(c, b, Ix);
  upload_img(c, d, Iy);
  Img cf = new_img(c, H, W, 7);
  F2 r = new_f2(c, H, W);
  flow_operator(c, op_args(P, alpha, 0.0), f, duv ? &df : nullptr, a, b, d, nullptr, cf, r);
  download_img(c, cf, coef);
  download_f2(c, r, rhs);
  HIPCHK(hipStreamSynchronize(c->stream));
  API_END(c)
}

int of_solve(of_ctx *c, const of_params *P, const float *coef, const float *rhs, int H, int W, float *x, int *iters,
             double *rel_residual) {
  API_BEGIN(c)
  REQUIRE(P && coef && rhs && x, OF_EINVAL, "bad arguments");
  check_params(P);
  Img cf = new_img(c, H, W, 7);
  upload_img(c, cf, coef);
  F2 b = upload_f2(c, rhs, H, W), xx = new_f2(c, H, W);
  SolveResult r = solve(c, P, cf, b, xx);
  download_f2(c, xx, x);
  HIPCHK(hipStreamSynchronize(c->stream));
  if (r.slot >= 0) {
    if (r.name) note_active(c, r.name, resolved(c, r.slot).iters + 1, r.px);
    r = resolved(c, r.slot);
  }
  if (iters) *iters = r.iters;
  if (rel_residual) *rel_residual = r.rel;
  API_END(c)
}

int of_flow_operator_dia(of_ctx *c, const of_params *P, double alpha, const float *uv, const float *duv,
                         const float *It, const float *Ix, const float *Iy, int H, int W, int nc, int *D_out,
                         float *planes, float *rhs) {
  API_BEGIN(c)
  REQUIRE(P && uv && It && Ix && Iy && planes && rhs && nc >= 1, OF_EINVAL, "bad arguments");
  REQUIRE(P->filters.general, OF_EINVAL, "of_flow_operator_dia needs params->filters.general");
  check_params(P);
  F2 f = upload_f2(c, uv, H, W);
  F2 df;
  if (duv) df = upload_f2(c, duv, H, W);
  Img a = new_img(c, H, W, nc), b = new_img(c, H, W, nc), d = new_img(c, H, W, nc);
  upload_img(c, a, It);
  upload_img(c, b, Ix);
  upload_img(c, d, Iy);
  GenLevel L = gen_level(c, P, H, W);
  F2 r = new_f2(c, H, W);
  gen_flow_operator(c, P, op_args(P, alpha, 0.0), f, duv ? &df : nullptr, a, b, d, nullptr, L, r);
  download_img(c, L.pl, planes);
  download_f2(c, r, rhs);
  HIPCHK(hipStreamSynchronize(c->stream));
  if (D_out) *D_out = L.D;
  API_END(c)
}
int of_solve_dia(of_ctx *c, const of_params *P, int D, const float *planes, const float *rhs, int H, int W, float *x,
                 int *iters, double *rel_residual) {
  API_BEGIN(c)
  REQUIRE(P && planes && rhs && x && D >= 0 && D <= GEN_MAXD, OF_EINVAL, "bad arguments");
  check_params(P);
  GenLevel L;
  L.D = D;
  L.pl = new_img(c, H, W, gen_nplanes(D));
  L.r = new_f2(c, H, W);
  L.p = new_f2(c, H, W);
  L.z = new_f2(c, H, W);
  L.q = new_f2(c, H, W);
  L.t = new_f2(c, H, W);
  L.e = new_f2(c, H, W);
  upload_img(c, L.pl, planes);
  F2 b = upload_f2(c, rhs, H, W), xx = new_f2(c, H, W);
  const SolveResult r = gen_solve_logged(c, P, L, b, xx);
  download_f2(c, xx, x);
  HIPCHK(hipStreamSynchronize(c->stream));
  if (iters) *iters = r.iters;
  if (rel_residual) *rel_residual = r.rel;
  API_END(c)
}
int of_detect_occlusion(of_ctx *c, const float *uv, const float *images, int H, int W, int nc, float *occ) {
  API_BEGIN(c)
  REQUIRE(uv && images && occ && nc >= 1, OF_EINVAL, "bad arguments");
  F2 f = upload_f2(c, uv, H, W), z = new_f2(c, H, W), u1 = new_f2(c, H, W);
  fill_f2(c, z, 0.0f);
  Img im = new_img(c, H, W, 2 * nc);
  upload_img(c, im, images);
  Img o = new_img(c, H, W, 1);
  Grid2 g = grid2(H, W);
  launch(c, "update_occ", k_update_occ, g.grid, g.block, 0, (const float2 *)f.p, (const float2 *)z.p, 0, u1.p,
         (const float *)im.p, (const float *)im.plane(nc), nc, o.p, H, W, f.P, im.ps());
  download_img(c, o, occ);
  HIPCHK(hipStreamSynchronize(c->stream));
  API_END(c)
}

int of_weighted_median(of_ctx *c, const float *uv, const float *guide, int gc, const float *occ, int H, int W,
                       int area_hsz, double sigma_i, float *out) {
  API_BEGIN(c)
  REQUIRE(uv && guide && occ && out && gc >= 1, OF_EINVAL, "bad arguments");
  F2 f = upload_f2(c, uv, H, W), o = new_f2(c, H, W);
  Img g = new_img(c, H, W, gc), oc = new_img(c, H, W, 1);
  upload_img(c, g, guide);
  upload_img(c, oc, occ);
  wmf(c, f, g, oc.p, o, area_hsz, sigma_i);
  download_f2(c, o, out);
  HIPCHK(hipStreamSynchronize(c->stream));
  API_END(c)
}

// flow_to_color (viz/flow_color.py:77-107): the wheel of make_colorwheel
// (flow_color.py:5-40) built on the host, the radius reduction and the
// per-pixel map on the device (k_flow_rad_max, k_flow_color)
}  // extern "C"
namespace {
ColorWheel color_wheel() {
  ColorWheel cw{};
  const int n[6] = {15, 6, 4, 11, 13, 6};
  // per segment: the channel held at 255, the ramped channel and whether it ramps down
  const int hold[6] = {0, 1, 1, 2, 2, 0}, ramp[6] = {1, 0, 2, 1, 0, 2};
  int k = 0;
  for (int s = 0; s < 6; ++s)
    for (int i = 0; i < n[s]; ++i, ++k) {
      const double r = std::floor(255.0 * i / n[s]);  // np.floor(255 * np.arange(n) / n)
      cw.w[3 * k + hold[s]] = 255;
      cw.w[3 * k + ramp[s]] = (unsigned char)(s % 2 ? 255.0 - r : r);
    }
  return cw;
}
template <typename T>
void flow_color_dev(of_ctx *c, const void *flow, long n, double fixed, uint8_t *out) {
  using U = typename OrdBits<T>::U;
  T *d = (T *)c->arena.alloc(sizeof(T) * 2 * n);
  U *mx = (U *)c->arena.alloc(sizeof(U));
  unsigned char *o = (unsigned char *)c->arena.alloc(3 * n);
  HIPCHK(hipMemcpyAsync(d, flow, sizeof(T) * 2 * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemsetAsync(mx, 0, sizeof(U), c->stream));
  const int blocks = (int)std::min<long>((n + 255) / 256, 2048);
  c->cur_px = (double)n;
  if (fixed <= 0) launch(c, "flow_rad_max", k_flow_rad_max<T>, dim3(blocks), dim3(256), 0, (const T *)d, n, mx);
  launch(c, "flow_color", k_flow_color<T>, dim3(blocks), dim3(256), 0, (const T *)d, n, (const U *)mx, fixed,
         color_wheel(), o);
  HIPCHK(hipMemcpyAsync(out, o, 3 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
}
}  // namespace
extern "C" {

int of_flow_to_color(of_ctx *c, const void *flow, int dtype, int H, int W, int has_max, double max_flow,
                     uint8_t *out_rgb) {
  API_BEGIN(c)
  REQUIRE(H >= 0 && W >= 0 && (dtype == 0 || dtype == 1) && (H * (long)W == 0 || (flow && out_rgb)), OF_EINVAL,
          "bad arguments");
  const long n = (long)H * W;
  // max_rad = max(max_flow, 1e-8) (flow_color.py:100): > 0 selects the fixed value
  const double fixed = has_max ? (max_flow > 1e-8 ? max_flow : 1e-8) : 0.0;
  if (n > 0) {
    if (dtype == 0) flow_color_dev<float>(c, flow, n, fixed, out_rgb);
    else flow_color_dev<double>(c, flow, n, fixed, out_rgb);
  }
  API_END(c)
}

int of_median_filter(of_ctx *c, const float *in, int H, int W, int planes, int size, float *out) {
  API_BEGIN(c)
  REQUIRE(in && out && planes >= 1, OF_EINVAL, "bad arguments");
  REQUIRE(size == 3 || size == 5 || size == 7, OF_ENOTSUP, "median size must be 3, 5 or 7");
  Img a = new_img(c, H, W, planes), b = new_img(c, H, W, planes);
  upload_img(c, a, in);
  Grid2 g = grid2(H, W);
  if (size == 3)
    launch(c, "median1", k_median1<3>, gz(g, planes), g.block, 0, (const float *)a.p, b.p, H, W, a.P, a.ps());
  else if (size == 5)
    launch(c, "median1", k_median1<5>, gz(g, planes), g.block, 0, (const float *)a.p, b.p, H, W, a.P, a.ps());
  else
    launch(c, "median1", k_median1<7>, gz(g, planes), g.block, 0, (const float *)a.p, b.p, H, W, a.P, a.ps());
  download_img(c, b, out);
  HIPCHK(hipStreamSynchronize(c->stream));
  API_END(c)
}

}  // extern "C"

#ifdef CGS_PHASE_TIMING
// instrumented builds only (tools/micro): read and clear the k_cgs role timers
extern "C" int of_debug_cgs_times(unsigned long long *out12) {
  if (hipMemcpyFromSymbol(out12, HIP_SYMBOL(g_cgs_t), sizeof(unsigned long long) * 12) != hipSuccess) return OF_EHIP;
  unsigned long long z[12] = {0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_cgs_t), z, sizeof(z)) != hipSuccess) return OF_EHIP;
  return OF_OK;
}
#endif
