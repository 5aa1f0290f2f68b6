// Per-phase timing of the weighted-median kernel at 1080p (Lab guide, h = 7):
// kernels_flow.hip built with WMF_PHASE_TIMING records clock64() at the phase
// boundaries of every wave; prints the mean cycles per phase and the launch time.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>
__device__ unsigned long long g_wmf_t[32400 * 8 + 64];
#include "kernels_flow.hip"
int main() {
  const int H = 1080, W = 1920, P = of_pitch(W), hsz = 7;
  const size_t ps = (size_t)H * P;
  std::vector<float> huv(2 * ps), hg(3 * ps), ho(ps);
  srand(1);
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < W; ++j) {
      size_t k = (size_t)i * P + j;
      huv[2 * k] = 2.f * sinf(6.2832f * i / H) + 0.5f + 0.05f * (rand() / (float)RAND_MAX - 0.5f);
      huv[2 * k + 1] = 1.5f * cosf(6.2832f * j / W) - 0.25f + 0.05f * (rand() / (float)RAND_MAX - 0.5f);
      for (int c = 0; c < 3; ++c) hg[c * ps + k] = 128.f + 60.f * sinf(0.05f * (i + 2 * j) + c) + 20.f * (rand() / (float)RAND_MAX);
      ho[k] = rand() / (float)RAND_MAX;
    }
  float2 *uv, *out; float *g, *o;
  hipMalloc(&uv, 2 * ps * 4); hipMalloc(&out, 2 * ps * 4); hipMalloc(&g, 3 * ps * 4); hipMalloc(&o, ps * 4);
  hipMemcpy(uv, huv.data(), 2 * ps * 4, hipMemcpyHostToDevice);
  hipMemcpy(g, hg.data(), 3 * ps * 4, hipMemcpyHostToDevice);
  hipMemcpy(o, ho.data(), ps * 4, hipMemcpyHostToDevice);
  const int RW = WMF_T + 2 * hsz, RP = RW + ((8 - RW) % 16 + 16) % 16, N = 512;
  const size_t shm = 2 * WMF_NC * 64 * sizeof(double) + (size_t)RW * RP * 16 + 2 * N * 2 + 2 * (size_t)RW * RP;
  dim3 grid(W / 8, (H + 7) / 8);
  const float nk = (float)(-1.4426950408889634 / (2.0 * 49.0));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_wmf<3, 8, 7>), grid, dim3(64), shm, 0, uv, g, o, out, H, W, P, ps, hsz, nk, RW, RP, (const float2 *)nullptr);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> t(32400 * 8);
    hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_wmf_t), t.size() * 8);
    double acc[6] = {0}; unsigned long long tmin = ~0ull, tmax = 0;
    const int nb = grid.x * grid.y;
    for (int b = 0; b < nb; ++b) {
      for (int i = 0; i < 5; ++i) acc[i] += (double)(t[b * 8 + i + 1] - t[b * 8 + i]);
      acc[5] += (double)(t[b * 8 + 5] - t[b * 8]);
      if (t[b * 8] < tmin) tmin = t[b * 8];
      if (t[b * 8 + 5] > tmax) tmax = t[b * 8 + 5];
    }
    printf("launch %.3f ms  shm %zu B  mean cycles per wave: load %.0f sort %.0f window %.0f chunk %.0f walk %.0f | total %.0f  (span %llu)\n",
           ms, shm, acc[0] / nb, acc[1] / nb, acc[2] / nb, acc[3] / nb, acc[4] / nb, acc[5] / nb, tmax - tmin);
  }
  return 0;
}
