// LDS scatter-add cost on gfx950: lane-private slots (c*64 + lane), c pseudo-random in [0,16),
// 450 updates per lane, 32400 one-wave blocks (the 1080p weighted-median grid).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
template <int MODE>
__global__ __launch_bounds__(64) void k(const unsigned *seed, float *out, int reps) {
  __shared__ double s[16 * 64 * 2];
  const int lane = threadIdx.x;
  for (int i = lane; i < 16 * 64 * 2; i += 64) s[i] = 0;
  __syncthreads();
  unsigned x = seed[blockIdx.x & 1023] ^ (lane * 2654435761u);
  float w = 1.0f + lane;
  for (int r = 0; r < reps; ++r) {
    x = x * 1664525u + 1013904223u;
    const int c = (x >> 28) & 15;
    if (MODE == 0) atomicAdd(&s[c * 64 + lane], (double)w);
    if (MODE == 1) atomicAdd(reinterpret_cast<unsigned long long *>(&s[c * 64 + lane]), (unsigned long long)x);
    if (MODE == 2) atomicAdd(reinterpret_cast<float *>(&s[c * 64 + lane]), w);
    if (MODE == 3) atomicAdd(reinterpret_cast<unsigned *>(&s[c * 64 + lane]), x);
    if (MODE == 4) s[c * 64 + lane] = (double)w;
    if (MODE == 5) reinterpret_cast<float *>(s)[c * 64 + lane] = w;
    w += 0.5f;
  }
  __syncthreads();
  out[blockIdx.x * 64 + lane] = (float)s[lane] + (float)s[lane + 64];
}
int main() {
  unsigned *seed; float *out;
  hipMalloc(&seed, 4096); hipMemset(seed, 7, 4096);
  const int nb = 32400; hipMalloc(&out, nb * 64 * 4);
  const char *names[] = {"ds_add_f64", "ds_add_u64", "ds_add_f32", "ds_add_u32", "ds_write_b64", "ds_write_b32"};
  void (*ks[])(const unsigned *, float *, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>};
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int m = 0; m < 6; ++m) {
    for (int reps : {0, 450}) {
      hipLaunchKernelGGL(ks[m], dim3(nb), dim3(64), 0, 0, seed, out, reps);
      hipEventRecord(a);
      for (int t = 0; t < 5; ++t) hipLaunchKernelGGL(ks[m], dim3(nb), dim3(64), 0, 0, seed, out, reps);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("%-13s reps %3d  %.3f ms/launch  -> %.2f LDS-cycles/instr/CU at 2.4GHz\n", names[m], reps, ms / 5,
             reps ? (ms / 5 * 1e-3 * 2.4e9) / ((double)nb / 256 * reps) : 0.0);
    }
  }
  return 0;
}
