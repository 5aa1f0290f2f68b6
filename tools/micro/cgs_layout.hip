// Placement sensitivity of the fused CG iteration (k_cgs) at 1080p: the same
// operator and vectors placed at different offsets inside one device buffer.
// The bench's 1080p solves run at two speeds (~38 and ~47 us per launch,
// profiles/r2u) depending on the GNC stage, i.e. on where the arena put that
// stage's buffers; this isolates placement from data.  Every launch reads
// the same r_in / p_old and a fixed partials record (alpha = 1, beta = 0.5),
// so timings are of identical work.
// usage: cgs_layout [seed-count]   (prints one JSON line per layout)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include "kernels_solve.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv) {
  const int nlay = argc > 1 ? atoi(argv[1]) : 12;
  const int H = 1080, W = 1920, P = of_pitch(W);
  const size_t ps = (size_t)H * P, vb = ps * 8;
  const size_t total = (size_t)1 << 30;  // 1 GiB pool
  char *pool;
  CK(hipMalloc(&pool, total));
  // host data: weights in [0.1, 1], diagonal = edge sums + data term
  std::vector<float> coef(ps * 7, 0.f), vec(ps * 2);
  srand(7);
  auto rnd = []() { return rand() / (float)RAND_MAX; };
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) {
      const size_t k = (size_t)i * P + j;
      for (int c = 0; c < 4; ++c) coef[c * ps + k] = 0.1f + 0.9f * rnd();
      if (j == W - 1) coef[0 * ps + k] = coef[2 * ps + k] = 0.f;
      if (i == H - 1) coef[1 * ps + k] = coef[3 * ps + k] = 0.f;
    }
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) {
      const size_t k = (size_t)i * P + j;
      float su = coef[k] + coef[ps + k], sv = coef[2 * ps + k] + coef[3 * ps + k];
      if (j > 0) { su += coef[k - 1]; sv += coef[2 * ps + k - 1]; }
      if (i > 0) { su += coef[ps + k - P]; sv += coef[3 * ps + k - P]; }
      const float g = rnd();
      coef[4 * ps + k] = su + g;
      coef[5 * ps + k] = 0.3f * g;
      coef[6 * ps + k] = sv + g;
    }
  for (auto &v : vec) v = rnd() - 0.5f;
  double *part, *part_w;
  PcgState *st;
  CK(hipMalloc(&part, sizeof(double) * 5 * PCG_MAX_BLOCKS));
  CK(hipMalloc(&part_w, sizeof(double) * 5 * PCG_MAX_BLOCKS));
  CK(hipMalloc(&st, sizeof(PcgState)));
  std::vector<double> hp(5 * PCG_MAX_BLOCKS, 0.0);
  hp[0 * PCG_MAX_BLOCKS] = 1.0;  // pq
  hp[1 * PCG_MAX_BLOCKS] = 0.5;  // qz
  hp[2 * PCG_MAX_BLOCKS] = 0.5;  // qMq
  hp[3 * PCG_MAX_BLOCKS] = 1.0;  // rz
  hp[4 * PCG_MAX_BLOCKS] = 1.0;  // rr
  CK(hipMemcpy(part, hp.data(), hp.size() * 8, hipMemcpyHostToDevice));
  // same geometry as the library (driver.hip cg_geometry, split = k_cgs)
  const int nstrips = (W + PCG_SWP - 1) / PCG_SWP;
  int nbands = std::max(1, std::min((H + 7) / 8, PCG_MAX_BLOCKS / nstrips));
  const int R = (H + nbands - 1) / nbands;
  nbands = (H + R - 1) / R;
  const float poly[6] = {5.4f, -9.5f, 10.9f, -7.7f, 3.1f, -0.55f};  // any fixed polynomial
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // buffers: coef, r0, r1, p0, p1, x, b
  srand(11);
  const size_t pads[6] = {1024, 4096, 65536, 262144, 1048576 + 4096, 3 * 1048576 + 12288};  // floats
  for (int lay = 0; lay < nlay + 6; ++lay) {
    const size_t cps = lay >= nlay ? ps + pads[lay - nlay] : ps;  // coefficient plane stride (floats)
    const size_t sz[7] = {cps * 7 * 4, vb, vb, vb, vb, vb, vb};
    size_t off[7];
    int order[7] = {0, 1, 2, 3, 4, 5, 6};
    if (lay == 0 || lay >= nlay) {  // packed in order, 256-B aligned (the arena's policy)
      size_t o = 0;
      for (int b = 0; b < 7; ++b) { off[b] = o; o += (sz[b] + 255) & ~(size_t)255; }
    } else {  // random order, random 256-B-aligned gaps up to 4 MiB
      for (int t = 6; t > 0; --t) std::swap(order[t], order[rand() % (t + 1)]);
      size_t o = (size_t)(rand() % 16384) * 256;
      for (int t = 0; t < 7; ++t) {
        const int b = order[t];
        off[b] = o;
        o += ((sz[b] + 255) & ~(size_t)255) + (size_t)(rand() % 16384) * 256;
      }
      if (o > total) { printf("{\"layout\": %d, \"skip\": true}\n", lay); continue; }
    }
    float *dc = (float *)(pool + off[0]);
    float2 *r0 = (float2 *)(pool + off[1]), *r1 = (float2 *)(pool + off[2]);
    float2 *p0 = (float2 *)(pool + off[3]), *p1 = (float2 *)(pool + off[4]);
    float2 *x = (float2 *)(pool + off[5]), *b = (float2 *)(pool + off[6]);
    for (int c = 0; c < 7; ++c) CK(hipMemcpy(dc + c * cps, coef.data() + c * ps, ps * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(r0, vec.data(), vb, hipMemcpyHostToDevice));
    CK(hipMemcpy(p0, vec.data(), vb, hipMemcpyHostToDevice));
    CK(hipMemcpy(x, vec.data(), vb, hipMemcpyHostToDevice));
    CK(hipMemcpy(b, vec.data(), vb, hipMemcpyHostToDevice));
    PcgArgs a;
    memset(&a, 0, sizeof(a));
    a.coef = dc; a.x = x; a.r_in = r0; a.p_old = p0; a.r_out = r1; a.p_new = p1; a.b = b;
    a.H = H; a.W = W; a.P = P; a.ps = cps; a.nb = nstrips * nbands;
    a.part_rd = part; a.part_wr = part_w; a.st = st; a.hflag = nullptr; a.rtol = 0.0; a.maxiter = 1 << 30;
    for (int i = 0; i < 6; ++i) a.poly[i] = poly[i];
    CK(hipMemset(st, 0, sizeof(PcgState)));
    const int reps = 60;
    float best = 1e9f, sum = 0.f;
    for (int r = 0; r < reps + 5; ++r) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL((k_cgs<false, false>), dim3(nstrips, nbands), dim3(64, 4), 0, 0, a, 5, R, nbands);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 5) { sum += ms; best = std::min(best, ms); }
    }
    printf("{\"layout\": %d, \"plane_pad_floats\": %zu, \"mean_us\": %.2f, \"best_us\": %.2f, \"off_MiB\": [", lay, cps - ps, sum / reps * 1e3, best * 1e3);
    for (int bb = 0; bb < 7; ++bb) printf("%s%.4f", bb ? ", " : "", off[bb] / 1048576.0);
    printf("], \"off_mod_2MiB_KiB\": [");
    for (int bb = 0; bb < 7; ++bb) printf("%s%.2f", bb ? ", " : "", (off[bb] % (2u << 20)) / 1024.0);
    printf("]}\n");
    fflush(stdout);
  }
  return 0;
}
