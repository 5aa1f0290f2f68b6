// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the
// optflow kernels use (4, 8, 16 B per lane): stream-read N bytes (sum into a
// per-block partial) and stream-write N bytes, one pass each, so the PMC
// counters can be compared with a known byte count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <typename T>
__global__ void rd(const T* __restrict__ a, size_t n, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float* f = reinterpret_cast<const float*>(&a[i]);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) s += f[k];
  }
  if (s == 12345.f) out[blockIdx.x] = s;
}

template <typename T>
__global__ void wr(T* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    T v;
    float* f = reinterpret_cast<float*>(&v);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) f[k] = (float)k;
    a[i] = v;
  }
}

int main() {
  const size_t bytes = (size_t)1 << 30;  // 1 GiB: 4x the MALL
  void* buf;
  float* out;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  hipMemset(buf, 0, bytes);
  const int grid = 256 * 8, block = 256;
  for (int rep = 0; rep < 2; ++rep) {
    rd<float><<<grid, block>>>((const float*)buf, bytes / 4, out);
    rd<float2><<<grid, block>>>((const float2*)buf, bytes / 8, out);
    rd<float4><<<grid, block>>>((const float4*)buf, bytes / 16, out);
    wr<float><<<grid, block>>>((float*)buf, bytes / 4);
    wr<float2><<<grid, block>>>((float2*)buf, bytes / 8);
    wr<float4><<<grid, block>>>((float4*)buf, bytes / 16);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("calib done: %zu bytes per dispatch\n", bytes);
  return 0;
}
