// Probe: v_mfma_f64_16x16x4f64 on gfx950 -- cycles per MFMA for one dependent accumulation
// chain (each MFMA's C is the previous D, the shape of mh_fullcov_kernel's row-block chains)
// against NA independent accumulators interleaved, at 1 and 2 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_f64_rate mfma_f64_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dbl4 __attribute__((ext_vector_type(4)));
#define N_ITER 2048

template <int NA>
__global__ void __launch_bounds__(256) probe(double* out, unsigned long long* cyc, double seed) {
  const int l = threadIdx.x & 63;
  double a = seed + l, b = 1.0 / (seed + l + 1);
  dbl4 e[NA];
  for (int i = 0; i < NA; ++i) e[i] = dbl4{0.0, 0.0, 0.0, 0.0};
  __syncthreads();
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
    for (int rep = 0; rep < 16 / NA; ++rep)
#pragma unroll
      for (int i = 0; i < NA; ++i) e[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e[i], 0, 0, 0);
    asm volatile("" : "+v"(a));
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  double s = 0;
  for (int i = 0; i < NA; ++i) s += e[i][0] + e[i][1] + e[i][2] + e[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NA>
void run(int waves_per_simd, double* out, unsigned long long* cyc) {
  const int block = 256 * waves_per_simd > 1024 ? 1024 : 256 * waves_per_simd;  // 4 waves = 1/SIMD
  for (int w = 0; w < 2; ++w) probe<NA><<<256, block>>>(out, cyc, 1.0 + w);
  hipDeviceSynchronize();
  unsigned long long h[256];
  hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < 256; ++i) m += (double)h[i];
  m /= 256;
  // per SIMD: waves_per_simd waves each ran 16 N_ITER MFMAs in m cycles
  printf("NA=%d waves/SIMD=%d  %.2f cycles per MFMA per SIMD (s_memtime clock)\n", NA,
         waves_per_simd, m / (16.0 * N_ITER * waves_per_simd));
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 1024 * 8);
  hipMalloc(&cyc, 256 * 8);
  for (int w = 1; w <= 2; ++w) {
    run<1>(w, out, cyc);
    run<2>(w, out, cyc);
    run<4>(w, out, cyc);
  }
  return 0;
}
