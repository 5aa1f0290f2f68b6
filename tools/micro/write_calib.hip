// WRITE_SIZE calibration for the assembly kernels' store pattern: NP fp32
// planes written with 4-B-per-lane stores (k_flow_operator / k_partial_deriv
// shape: 64x4 blocks, grid-stride over rows) vs 16-B-per-lane stores (4 px
// per thread), 1920x1080, pitch 1920.  Bytes written per launch are printed;
// run under rocprofv3 --pmc WRITE_SIZE.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int NP>
__global__ void k_dword(float *out, int H, int W, size_t ps) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  for (int i = blockIdx.y * 4 + threadIdx.y; i < H; i += gridDim.y * 4) {
    const size_t k = (size_t)i * W + j;
#pragma unroll
    for (int p = 0; p < NP; ++p) out[p * ps + k] = (float)(i + j + p);
  }
}
template <int NP>
__global__ void k_vec4(float4 *out, int H, int W4, size_t ps4) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  for (int i = blockIdx.y * 4 + threadIdx.y; i < H; i += gridDim.y * 4) {
    const size_t k = (size_t)i * W4 + j;
    if (j < W4)
#pragma unroll
      for (int p = 0; p < NP; ++p) out[p * ps4 + k] = make_float4(i, j, p, 1.f);
  }
}
int main() {
  const int H = 1080, W = 1920;
  const size_t ps = (size_t)H * W;
  float *buf;
  hipMalloc(&buf, 8 * ps * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
    hipEventRecord(a);
    hipLaunchKernelGGL(k_dword<8>, dim3(W / 64, 68), dim3(64, 4), 0, 0, buf, H, W, ps);
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    printf("dword x8 planes: %.1f MB, %.1f us\n", 8 * ps * 4 / 1e6, ms * 1e3);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_dword<3>, dim3(W / 64, 68), dim3(64, 4), 0, 0, buf, H, W, ps);
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    printf("dword x3 planes: %.1f MB, %.1f us\n", 3 * ps * 4 / 1e6, ms * 1e3);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_vec4<8>, dim3((W / 4 + 63) / 64, 68), dim3(64, 4), 0, 0, (float4 *)buf, H, W / 4, ps / 4);
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    printf("vec4  x8 planes: %.1f MB, %.1f us\n", 8 * ps * 4 / 1e6, ms * 1e3);
  }
  return 0;
}
