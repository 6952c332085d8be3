// Probe: numerics of v_mfma_f64_16x16x4f64 on gfx950 -- is D = fma-chain over k (k ascending,
// C first)?  Writes A, B, C, D for random inputs; scripts/probes/mfma_f64_check.py compares.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef double double4_t __attribute__((ext_vector_type(4)));

__global__ void k(const double* A, const double* B, const double* C, double* D, int reps) {
  const int l = threadIdx.x;
  for (int r = 0; r < reps; ++r) {
    // A[i][k]: lane l -> i = l % 16, k = l / 16 ; B[k][j]: lane l -> k = l / 16, j = l % 16
    const double a = A[r * 64 + (l % 16) * 4 + l / 16];
    const double b = B[r * 64 + (l / 16) * 16 + l % 16];
    double4_t c;
    for (int q = 0; q < 4; ++q) c[q] = C[r * 256 + ((l >> 4) + 4 * q) * 16 + (l & 15)];
    double4_t d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int q = 0; q < 4; ++q) D[r * 256 + ((l >> 4) + 4 * q) * 16 + (l & 15)] = d[q];
  }
}

int main(int argc, char** argv) {
  const int reps = 4096;
  std::mt19937_64 g(1);
  std::vector<double> A(reps * 64), B(reps * 64), C(reps * 256), D(reps * 256);
  auto rnd = [&]() {
    // wide exponent spread so that rounding order shows
    double m = std::ldexp((double)(g() >> 11), -53) * 2 - 1;
    int e = (int)(g() % 60) - 30;
    return std::ldexp(m, e);
  };
  for (auto& v : A) v = rnd();
  for (auto& v : B) v = rnd();
  for (auto& v : C) v = rnd();
  double *dA, *dB, *dC, *dD;
  hipMalloc(&dA, A.size() * 8); hipMalloc(&dB, B.size() * 8); hipMalloc(&dC, C.size() * 8); hipMalloc(&dD, D.size() * 8);
  hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, reps);
  hipMemcpy(D.data(), dD, D.size() * 8, hipMemcpyDeviceToHost);
  FILE* f = fopen(argc > 1 ? argv[1] : "mfma_probe.bin", "wb");
  fwrite(A.data(), 8, A.size(), f); fwrite(B.data(), 8, B.size(), f);
  fwrite(C.data(), 8, C.size(), f); fwrite(D.data(), 8, D.size(), f);
  fclose(f);
  printf("probe done reps=%d\n", reps);
  return 0;
}
