// Probe: do f64 MFMAs and f64 VALU FMAs of two waves on one SIMD run concurrently on gfx950?
// 512-thread workgroups (two waves per SIMD): waves 0-3 issue v_mfma_f64_16x16x4f64 (four
// independent accumulators), waves 4-7 issue v_fma_f64 (eight independent chains).  Mode 1: MFMA
// waves only; 2: VALU waves only; 3: both.  Cycles (s_memtime) per loop of each role.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_valu_overlap mfma_valu_overlap.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dbl4 __attribute__((ext_vector_type(4)));
#define N_ITER 4096

__global__ void __launch_bounds__(512) probe(double* out, unsigned long long* cyc, int mode, double seed) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const bool mf = w < 4;
  double a = seed + l, b = 1.0 / (seed + l + 1);
  double s = 0.0;
  __syncthreads();
  const unsigned long long t0 = __builtin_readcyclecounter();
  if (mf && (mode & 1)) {
    dbl4 e0 = {0, 0, 0, 0}, e1 = e0, e2 = e0, e3 = e0;
    for (int it = 0; it < N_ITER; ++it) {
      e0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e0, 0, 0, 0);
      e1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e1, 0, 0, 0);
      e2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e2, 0, 0, 0);
      e3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e3, 0, 0, 0);
      asm volatile("" : "+v"(a));
    }
    s = e0[0] + e1[1] + e2[2] + e3[3];
  } else if (!mf && (mode & 2)) {
    double v[8];
    for (int i = 0; i < 8; ++i) v[i] = a + i;
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fma(v[i], b, a);
      asm volatile("" : "+v"(a));
    }
    for (int i = 0; i < 8; ++i) s += v[i];
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 512 * 8);
  hipMalloc(&cyc, 256 * 8 * 8);
  for (int mode = 1; mode <= 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) probe<<<256, 512>>>(out, cyc, mode, 1.0 + rep);
    hipDeviceSynchronize();
    unsigned long long h[256 * 8];
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    double m = 0, v = 0;
    for (int b = 0; b < 256; ++b) {
      for (int w = 0; w < 4; ++w) m += (double)h[b * 8 + w];
      for (int w = 4; w < 8; ++w) v += (double)h[b * 8 + w];
    }
    m /= 1024.0;
    v /= 1024.0;
    printf("mode %d: MFMA waves %.1f cycles per MFMA (4 per iter), VALU waves %.2f cycles per v_fma_f64\n",
           mode, m / (4.0 * N_ITER), v / (32.0 * N_ITER));
  }
  return 0;
}
