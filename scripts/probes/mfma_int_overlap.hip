// Probe: which VALU work runs beside the f64 matrix core on gfx950?  (C5's step issues 40
// v_mfma_f64_16x16x4f64 and ~600 VALU per 16 chain-steps; f64 VALU FMAs keep only 0.374 of their
// rate beside an MFMA, scripts/probes/mfma_valu_overlap.hip.)  512-thread workgroups, two waves
// per SIMD.  Modes:
//   1  waves 0-3: MFMAs (4 independent accumulators per iteration)            waves 4-7 idle
//   2  waves 4-7: Philox-like int32 VALU (v_mul_hi/lo_u32 + xor, 8 chains)      waves 0-3 idle
//   3  both roles at once (separate waves)
//   4  waves 0-3: per iteration 4 MFMAs AND the int work of mode 2 (one wave issues both)
//   5  waves 0-3: per iteration 4 MFMAs AND 32 f64 FMAs (one wave issues both)
// Prints cycles per iteration of each role (s_memtime / readcyclecounter).
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_int_overlap mfma_int_overlap.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dbl4 __attribute__((ext_vector_type(4)));
#define N_ITER 2048

__device__ __forceinline__ void int_work(unsigned* v, unsigned k) {
#pragma unroll
  for (int i = 0; i < 8; i += 2) {               // one Philox round on 4 chains of pairs
    const unsigned hi = __umulhi(0xD2511F53u, v[i]), lo = 0xD2511F53u * v[i];
    v[i] = hi ^ v[i + 1] ^ k;
    v[i + 1] = lo;
  }
}

__global__ void __launch_bounds__(512) probe(double* out, unsigned long long* cyc, int mode, double seed) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const bool mf = w < 4;
  double a = seed + l, b = 1.0 / (seed + l + 1);
  double s = 0.0;
  unsigned v[8];
  for (int i = 0; i < 8; ++i) v[i] = 0x9E3779B9u * (l + i + 1);
  double f[8];
  for (int i = 0; i < 8; ++i) f[i] = a + i;
  __syncthreads();
  const unsigned long long t0 = __builtin_readcyclecounter();
  if (mf && (mode == 1 || mode == 3 || mode == 4 || mode == 5)) {
    dbl4 e0 = {0, 0, 0, 0}, e1 = e0, e2 = e0, e3 = e0;
    for (int it = 0; it < N_ITER; ++it) {
      e0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e0, 0, 0, 0);
      if (mode == 4) { int_work(v, it); int_work(v, it + 1); }
      if (mode == 5) {
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = fma(f[i], b, a);
      }
      e1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e1, 0, 0, 0);
      if (mode == 4) { int_work(v, it + 2); int_work(v, it + 3); }
      if (mode == 5) {
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = fma(f[i], b, a);
      }
      e2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e2, 0, 0, 0);
      if (mode == 4) { int_work(v, it + 4); int_work(v, it + 5); }
      if (mode == 5) {
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = fma(f[i], b, a);
      }
      e3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e3, 0, 0, 0);
      if (mode == 4) { int_work(v, it + 6); int_work(v, it + 7); }
      if (mode == 5) {
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = fma(f[i], b, a);
      }
      asm volatile("" : "+v"(a));
    }
    s = e0[0] + e1[1] + e2[2] + e3[3];
  } else if (!mf && (mode == 2 || mode == 3)) {
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
      for (int r = 0; r < 8; ++r) int_work(v, it + r);
    }
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  for (int i = 0; i < 8; ++i) s += (double)v[i] + f[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 512 * 8);
  hipMalloc(&cyc, 256 * 8 * 8);
  for (int mode = 1; mode <= 5; ++mode) {
    for (int rep = 0; rep < 2; ++rep) probe<<<256, 512>>>(out, cyc, mode, 1.0 + rep);
    hipDeviceSynchronize();
    unsigned long long h[256 * 8];
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    double m = 0, v = 0;
    for (int b = 0; b < 256; ++b) {
      for (int w = 0; w < 4; ++w) m += (double)h[b * 8 + w];
      for (int w = 4; w < 8; ++w) v += (double)h[b * 8 + w];
    }
    m /= 1024.0 * N_ITER;
    v /= 1024.0 * N_ITER;
    printf("mode %d: waves 0-3 %.1f cycles/iter, waves 4-7 %.1f cycles/iter\n", mode, m, v);
  }
  return 0;
}
