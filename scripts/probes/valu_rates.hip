// Issue-rate probe for the VALU instructions on the MH step's critical mix (gfx950):
// 8 independent chains per lane of one instruction, 16 waves per CU, timed with hipEvents.
// Prints cycles per wave-instruction per SIMD at the assumed clock (relative costs are what
// matter: v_add_u32 is the full-rate reference).
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_ITER 8192

#define CHAIN8(ASM, T, C)                                                     \
  _Pragma("unroll 4") for (int it = 0; it < N_ITER; ++it) {                                   \
    asm volatile(ASM : "+" C(r0) : "s"(kk) : "vcc");                                          \
    asm volatile(ASM : "+" C(r1) : "s"(kk) : "vcc");                                          \
    asm volatile(ASM : "+" C(r2) : "s"(kk) : "vcc");                                          \
    asm volatile(ASM : "+" C(r3) : "s"(kk) : "vcc");                                          \
    asm volatile(ASM : "+" C(r4) : "s"(kk) : "vcc");                                          \
    asm volatile(ASM : "+" C(r5) : "s"(kk) : "vcc");                                          \
    asm volatile(ASM : "+" C(r6) : "s"(kk) : "vcc");                                          \
    asm volatile(ASM : "+" C(r7) : "s"(kk) : "vcc");                                          \
  }

template <int OP>
__global__ void __launch_bounds__(256) probe(double* out, uint32_t seed) {
  const uint32_t t = threadIdx.x + blockIdx.x * 256 + seed;
  const uint32_t kk = 0xD2511F53u ^ (seed & 1);
  if constexpr (OP < 100) {
    // 32-bit register ops
    uint32_t r0 = t, r1 = t + 1, r2 = t + 2, r3 = t + 3, r4 = t + 4, r5 = t + 5, r6 = t + 6, r7 = t + 7;
    if constexpr (OP == 0) CHAIN8("v_add_u32 %0, %0, %1", uint32_t, "v")
    if constexpr (OP == 1) CHAIN8("v_mul_hi_u32 %0, %0, %1", uint32_t, "v")
    if constexpr (OP == 2) CHAIN8("v_mul_lo_u32 %0, %0, %1", uint32_t, "v")
    if constexpr (OP == 3) CHAIN8("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96", uint32_t, "v")
    if constexpr (OP == 4) CHAIN8("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", uint32_t, "v")
    if constexpr (OP == 5) CHAIN8("v_mul_u32_u24 %0, %0, %1", uint32_t, "v")
    if constexpr (OP == 6) CHAIN8("v_fma_f32 %0, %0, %0, 1.0", float, "v")
    if constexpr (OP == 7) CHAIN8("v_ffbh_u32 %0, %0", uint32_t, "v")
    out[t] = (double)(r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7);
  } else {
    // 64-bit register ops
    double r0 = t, r1 = t + 1, r2 = t + 2, r3 = t + 3, r4 = t + 4, r5 = t + 5, r6 = t + 6, r7 = t + 7;
    if constexpr (OP == 100) CHAIN8("v_fma_f64 %0, %0, %0, 1.0", double, "v")
    if constexpr (OP == 101) CHAIN8("v_mul_f64 %0, %0, 0.5", double, "v")
    if constexpr (OP == 102) CHAIN8("v_add_f64 %0, %0, 1.0", double, "v")
    if constexpr (OP == 103) {
      uint32_t vin = t * 3u;
      _Pragma("unroll 4") for (int it = 0; it < N_ITER; ++it) {
#define MADU(R) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(R) : "s"(kk), "v"(vin) : "vcc");
        MADU(r0) MADU(r1) MADU(r2) MADU(r3) MADU(r4) MADU(r5) MADU(r6) MADU(r7)
      }
    }
    if constexpr (OP == 104) CHAIN8("v_ldexp_f64 %0, %0, 3", double, "v")
    if constexpr (OP == 105) CHAIN8("v_rsq_f64 %0, %0", double, "v")
    if constexpr (OP == 106) CHAIN8("v_pk_fma_f32 %0, %0, %0, %0", double, "v")
    if constexpr (OP == 107) CHAIN8("v_mov_b64 %0, %0", double, "v")
    if constexpr (OP == 108) CHAIN8("v_cvt_f64_u32 %0, %1", double, "v")
    if constexpr (OP == 109) CHAIN8("v_lshl_add_u64 %0, %0, 3, %0", double, "v")
    out[t] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
  }
}

template <int OP>
void run(const char* name, double* out, hipEvent_t e0, hipEvent_t e1) {
  const int waves_per_cu = 16, cus = 256;
  const int blocks = cus * waves_per_cu / 4;
  probe<OP><<<blocks, 256>>>(out, 1);   // warm
  hipEventRecord(e0);
  for (int rep = 0; rep < 5; ++rep) probe<OP><<<blocks, 256>>>(out, rep);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double instr_per_wave = 8.0 * N_ITER * 5;
  const double waves_per_simd = waves_per_cu / 4.0;
  const double cyc = ms * 1e-3 * 2.4e9 / (waves_per_simd * instr_per_wave);
  printf("%-16s %8.3f ms  %6.2f cycles/wave-instr/SIMD @2.4GHz\n", name, ms, cyc);
}

int main() {
  double* out;
  hipMalloc(&out, 256 * 16 * 64 * 8 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  run<0>("v_add_u32", out, e0, e1);
  run<1>("v_mul_hi_u32", out, e0, e1);
  run<2>("v_mul_lo_u32", out, e0, e1);
  run<3>("v_bitop3_b32", out, e0, e1);
  run<4>("v_mov_b32_dpp", out, e0, e1);
  run<5>("v_mul_u32_u24", out, e0, e1);
  run<6>("v_fma_f32", out, e0, e1);
  run<7>("v_ffbh_u32", out, e0, e1);
  run<100>("v_fma_f64", out, e0, e1);
  run<101>("v_mul_f64", out, e0, e1);
  run<102>("v_add_f64", out, e0, e1);
  run<103>("v_mad_u64_u32", out, e0, e1);
  run<104>("v_ldexp_f64", out, e0, e1);
  run<105>("v_rsq_f64", out, e0, e1);
  run<106>("v_pk_fma_f32", out, e0, e1);
  run<107>("v_mov_b64", out, e0, e1);
  run<108>("v_cvt_f64_u32", out, e0, e1);
  run<109>("v_lshl_add_u64", out, e0, e1);
  return 0;
}
