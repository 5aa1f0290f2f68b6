// Issue cost of the vector instructions the weighted-median kernel (k_wmf)
// is made of, on gfx950: each case runs 32 independent instructions of one
// opcode per loop step (8 register chains, so no result is read within 8
// instructions of being written), REPS steps, timed with s_memtime inside the
// wave.  Printed: wave-cycles per instruction with 1 wave per SIMD and with 2
// (the weighted median's occupancy), i.e. the price tools/isa_census.py puts on
// each opcode class.  Build: hipcc --offload-arch=gfx950 -O3 valu_cost.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REPS 256
#define X8(s) s s s s s s s s

// 8 chains of 32-bit (f) / 64-bit (d) operands; OPS is one asm template over
// %0..%7 (chains) and %8 (a shared source), repeated twice per step
#define CASE32(name, ins)                                                                          \
  __global__ __launch_bounds__(64) void k_##name(float *out, unsigned long long *cyc, float seed) { \
    float a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5,     \
          a6 = seed + 6, a7 = seed + 7, c = seed * 0.5f;                                           \
    const unsigned long long t0 = clock64();                                                        \
    for (int r = 0; r < REPS; ++r)                                                                 \
      asm volatile(ins ins ins ins : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                   "+v"(a7) : "v"(c) : "v40", "v41", "s0", "s1", "vcc");                                                             \
    const unsigned long long t1 = clock64();                                                        \
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                    \
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                               \
  }
#define CASE64(name, ins)                                                                           \
  __global__ __launch_bounds__(64) void k_##name(float *out, unsigned long long *cyc, float seed) {  \
    double a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5,     \
           a6 = seed + 6, a7 = seed + 7, c = seed * 0.5;                                            \
    const unsigned long long t0 = clock64();                                                         \
    for (int r = 0; r < REPS; ++r)                                                                  \
      asm volatile(ins ins ins ins : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),  \
                   "+v"(a7) : "v"(c) : "v40", "v41", "s0", "s1", "vcc");                                                              \
    const unsigned long long t1 = clock64();                                                         \
    out[blockIdx.x * 64 + threadIdx.x] = (float)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);            \
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                                \
  }
#define ALL8(op) op(0) op(1) op(2) op(3) op(4) op(5) op(6) op(7)
#define S(x) #x
#define F_ADD(i) "v_add_f32 %" S(i) ", %" S(i) ", %8\n"
#define F_MUL(i) "v_mul_f32 %" S(i) ", %" S(i) ", %8\n"
#define F_FMA(i) "v_fmac_f32 %" S(i) ", %" S(i) ", %8\n"
#define F_EXP(i) "v_exp_f32 %" S(i) ", %" S(i) "\n"
#define F_MAX(i) "v_max_f32 %" S(i) ", %" S(i) ", %8\n"
#define F_AND(i) "v_and_b32 %" S(i) ", %" S(i) ", %8\n"
#define F_BFE(i) "v_bfe_u32 %" S(i) ", %" S(i) ", 8, 8\n"
#define F_LSA(i) "v_lshl_add_u32 %" S(i) ", %" S(i) ", 9, %8\n"
#define F_CND(i) "v_cndmask_b32 %" S(i) ", %" S(i) ", %8, vcc\n"
#define F_CND3(i) "v_cndmask_b32_e64 %" S(i) ", %" S(i) ", %8, s[0:1]\n"
#define F_DPP(i) "v_mov_b32_dpp %" S(i) ", %" S(i) " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define F_DPPR(i) "v_mov_b32_dpp %" S(i) ", %" S(i) " row_ror:8 row_mask:0xf bank_mask:0xf\n"
#define F_XOR(i) "v_xor_b32 %" S(i) ", 0x80000000, %" S(i) "\n"
#define F_MULLO(i) "v_mul_lo_u32 %" S(i) ", %" S(i) ", %8\n"
#define F_SDWA(i) "v_sub_u32_sdwa %" S(i) ", %" S(i) ", %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\n"
#define F_CVT(i) "v_cvt_f64_f32 v[40:41], %" S(i) "\n"
#define D_MIN(i) "v_min_f64 %" S(i) ", %" S(i) ", %8\n"
#define D_MINN(i) "v_min_f64 %" S(i) ", %" S(i) ", -%8\n"
#define D_ADD(i) "v_add_f64 %" S(i) ", %" S(i) ", %8\n"
#define D_CMP(i) "v_cmp_nlt_f64_e64 s[0:1], %" S(i) ", %8\n"
#define D_CMPV(i) "v_cmp_nlt_f64 vcc, %" S(i) ", %8\n"
#define D_LSH(i) "v_lshl_add_u64 %" S(i) ", %" S(i) ", 0, %8\n"
#define D_MOV(i) "v_mov_b64 %" S(i) ", %8\n"
#define D_PKADD(i) "v_pk_add_f32 %" S(i) ", %" S(i) ", %8\n"
#define D_PKMUL(i) "v_pk_mul_f32 %" S(i) ", %" S(i) ", %8\n"
#define D_PKFMA(i) "v_pk_fma_f32 %" S(i) ", %" S(i) ", %8, %" S(i) "\n"
#define F_SWAP4 "v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3\n v_permlane32_swap_b32 %4, %5\n v_permlane32_swap_b32 %6, %7\n"

CASE32(add_f32, ALL8(F_ADD))
CASE32(mul_f32, ALL8(F_MUL))
CASE32(fmac_f32, ALL8(F_FMA))
CASE32(exp_f32, ALL8(F_EXP))
CASE32(max_f32, ALL8(F_MAX))
CASE32(and_b32, ALL8(F_AND))
CASE32(bfe_u32, ALL8(F_BFE))
CASE32(lshl_add_u32, ALL8(F_LSA))
CASE32(cndmask_vcc, ALL8(F_CND))
CASE32(cndmask_e64, ALL8(F_CND3))
CASE32(dpp_quad, ALL8(F_DPP))
CASE32(dpp_row_ror, ALL8(F_DPPR))
CASE32(xor_b32, ALL8(F_XOR))
CASE32(cvt_f64_f32, ALL8(F_CVT))
CASE32(mul_lo_u32, ALL8(F_MULLO))
CASE32(sub_u32_sdwa, ALL8(F_SDWA))
CASE64(min_f64, ALL8(D_MIN))
CASE64(min_f64_neg, ALL8(D_MINN))
CASE64(add_f64, ALL8(D_ADD))
CASE64(cmp_f64_sgpr, ALL8(D_CMP))
CASE64(cmp_f64_vcc, ALL8(D_CMPV))
CASE64(lshl_add_u64, ALL8(D_LSH))
CASE64(mov_b64, ALL8(D_MOV))
CASE64(pk_add_f32, ALL8(D_PKADD))
CASE64(pk_mul_f32, ALL8(D_PKMUL))
CASE64(pk_fma_f32, ALL8(D_PKFMA))
CASE32(permlane32_swap, F_SWAP4 F_SWAP4)

typedef void (*kfn)(float *, unsigned long long *, float);
struct Case {
  const char *name;
  kfn k;
};
int main() {
  const Case cases[] = {
      {"v_add_f32", k_add_f32},          {"v_mul_f32", k_mul_f32},          {"v_fmac_f32", k_fmac_f32},
      {"v_exp_f32", k_exp_f32},          {"v_max_f32", k_max_f32},          {"v_and_b32", k_and_b32},
      {"v_bfe_u32", k_bfe_u32},          {"v_lshl_add_u32", k_lshl_add_u32}, {"v_cndmask_b32(vcc)", k_cndmask_vcc},
      {"v_cndmask_b32_e64", k_cndmask_e64}, {"v_mov_b32_dpp quad_perm", k_dpp_quad},
      {"v_mov_b32_dpp row_ror", k_dpp_row_ror}, {"v_xor_b32", k_xor_b32}, {"v_cvt_f64_f32", k_cvt_f64_f32},
      {"v_mul_lo_u32", k_mul_lo_u32},    {"v_sub_u32_sdwa", k_sub_u32_sdwa},
      {"v_min_f64", k_min_f64},          {"v_min_f64 (neg src)", k_min_f64_neg}, {"v_add_f64", k_add_f64},
      {"v_cmp_nlt_f64_e64", k_cmp_f64_sgpr}, {"v_cmp_nlt_f64(vcc)", k_cmp_f64_vcc},
      {"v_lshl_add_u64", k_lshl_add_u64}, {"v_mov_b64", k_mov_b64},        {"v_pk_add_f32", k_pk_add_f32},
      {"v_pk_mul_f32", k_pk_mul_f32},    {"v_pk_fma_f32", k_pk_fma_f32},    {"v_permlane32_swap", k_permlane32_swap},
  };
  float *out;
  unsigned long long *cyc;
  hipMalloc(&out, 2048 * 64 * 4);
  hipMalloc(&cyc, 2048 * 8);
  unsigned long long h[2048];
  printf("{\"unit\": \"wave-cycles per instruction (s_memtime), 32 independent per step, %d steps\", \"cases\": [\n", REPS);
  const int n = sizeof(cases) / sizeof(cases[0]);
  for (int i = 0; i < n; ++i) {
    double res[2];
    // 1 wave per SIMD: 4 one-wave blocks per CU x 256 CUs (1024 blocks); 2
    // per SIMD: 2048 blocks (the grid fills every SIMD evenly either way)
    const int nbs[2] = {1024, 2048};
    for (int m = 0; m < 2; ++m) {
      hipLaunchKernelGGL(cases[i].k, dim3(nbs[m]), dim3(64), 0, 0, out, cyc, 1.0f);  // warm
      hipLaunchKernelGGL(cases[i].k, dim3(nbs[m]), dim3(64), 0, 0, out, cyc, 1.0f);
      hipMemcpy(h, cyc, nbs[m] * 8, hipMemcpyDeviceToHost);
      double s = 0;
      for (int b = 0; b < nbs[m]; ++b) s += (double)h[b];
      res[m] = s / nbs[m] / (32.0 * REPS);
    }
    printf("  {\"op\": \"%s\", \"w1\": %.2f, \"w2\": %.2f}%s\n", cases[i].name, res[0], res[1], i + 1 < n ? "," : "");
  }
  printf("]}\n");
  return 0;
}
