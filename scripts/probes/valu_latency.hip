// Dependent-issue latency probe (gfx950): ONE dependency chain per lane, one wave per SIMD, so
// every instruction waits for its predecessor.  cycles/instr = s_memtime delta / chain length.
// Compared with valu_rates (8 independent chains, many waves: issue rate), this shows how much
// instruction-level parallelism a wave needs to keep its SIMD busy on each instruction class.
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_ITER 4096

#define DEP(ASM, C)                                                              \
  for (int it = 0; it < N_ITER; ++it) {                                          \
    asm volatile(ASM : "+" C(r0) : "s"(kk) : "vcc");                             \
    asm volatile(ASM : "+" C(r0) : "s"(kk) : "vcc");                             \
    asm volatile(ASM : "+" C(r0) : "s"(kk) : "vcc");                             \
    asm volatile(ASM : "+" C(r0) : "s"(kk) : "vcc");                             \
  }

template <int OP>
__global__ void __launch_bounds__(64) probe(double* out, unsigned long long* cyc, uint32_t seed) {
  __shared__ double lds[4096];
  const uint32_t t = threadIdx.x + seed;
  for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = 0.0;
  __syncthreads();
  const uint32_t kk = 0xD2511F53u ^ (seed & 1);
  unsigned long long t0 = __builtin_readcyclecounter();
  double res = 0;
  if constexpr (OP < 100) {
    uint32_t r0 = t;
    if constexpr (OP == 0) DEP("v_add_u32 %0, %0, %1", "v")
    if constexpr (OP == 1) DEP("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96", "v")
    if constexpr (OP == 2) DEP("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", "v")
    if constexpr (OP == 3) DEP("v_mul_hi_u32 %0, %0, %1", "v")
    res = r0;
  } else if constexpr (OP < 200) {
    double r0 = t;
    if constexpr (OP == 100) DEP("v_fma_f64 %0, %0, %0, 1.0", "v")
    if constexpr (OP == 101) DEP("v_add_f64 %0, %0, 1.0", "v")
    if constexpr (OP == 102) {
      uint32_t vin = t * 3u;
      for (int it = 0; it < N_ITER; ++it) {
#define MADU asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(r0) : "s"(kk), "v"(vin) : "vcc");
        MADU MADU MADU MADU
      }
    }
    if constexpr (OP == 103) {
      // mad_u64 whose 32-bit input is the previous result's high half (the Philox round shape)
      uint32_t a = t;
      for (int it = 0; it < 4 * N_ITER; ++it) {
        uint64_t p;
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p) : "v"(a), "s"(kk) : "vcc");
        a = (uint32_t)(p >> 32);
      }
      r0 = a;
    }
    res = r0;
  } else {
    // LDS read latency: pointer chase through lds (address from the previous read)
    uint32_t a = (t & 63) * 16;
    for (int it = 0; it < 4 * N_ITER; ++it) {
      double4 v;
      if constexpr (OP == 200) {
        double2 q;
        asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(q) : "v"(a));
        a = a + (uint32_t)__double2loint(q.x);
      } else {
        double q;
        asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(q) : "v"(a));
        a = a + (uint32_t)__double2loint(q);
      }
      (void)v;
    }
    res = a;
  }
  unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * 64 + threadIdx.x] = res;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char* name, double* out, unsigned long long* cyc) {
  probe<OP><<<256, 64>>>(out, cyc, 1);
  hipDeviceSynchronize();
  probe<OP><<<256, 64>>>(out, cyc, 2);
  hipDeviceSynchronize();
  unsigned long long h[256];
  hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
  unsigned long long m = 0;
  for (int i = 0; i < 256; ++i) m += h[i];
  printf("%-22s %7.2f cycles per dependent instruction (s_memtime clock)\n", name,
         (double)m / 256 / (4.0 * N_ITER));
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 64 * 8);
  hipMalloc(&cyc, 256 * 8);
  run<0>("v_add_u32", out, cyc);
  run<1>("v_bitop3_b32", out, cyc);
  run<2>("v_mov_b32_dpp", out, cyc);
  run<3>("v_mul_hi_u32", out, cyc);
  run<100>("v_fma_f64", out, cyc);
  run<101>("v_add_f64", out, cyc);
  run<102>("v_mad_u64_u32 (acc)", out, cyc);
  run<103>("v_mad_u64_u32 (hi->in)", out, cyc);
  run<200>("ds_read_b128+wait", out, cyc);
  run<201>("ds_read_b64+wait", out, cyc);
  return 0;
}
