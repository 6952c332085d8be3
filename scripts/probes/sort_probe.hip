// Microbenchmark of the one-workgroup bitonic network used for the nested new-key sort
// (mcg_nested_kernels.hip): full network vs load/store only, k = 4096.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ bool nk_less(double la, int ja, double lb, int jb) {
  return la < lb || (la == lb && ja > jb);
}

template <int MODE>
__global__ void __launch_bounds__(1024) sort_k(const double* in, double* out, int* oj, int k, int L) {
  __shared__ double sl[4096];
  __shared__ int sj[4096];
  const int t = threadIdx.x;
  double kl[4];
  int kj[4];
  for (int e = 0; e < 4; ++e) {
    const int p = 4 * t + e;
    kl[e] = p < k ? in[p] : __builtin_inf();
    kj[e] = p < k ? p : -1;
  }
  auto sel = [](double& l, int& j, double ol, int ojv, bool keep_min) {
    const bool other_less = nk_less(ol, ojv, l, j);
    if (other_less == keep_min) { l = ol; j = ojv; }
  };
  if (MODE == 1) {
    for (int size = 2; size <= L; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        if (stride <= 2) {
          for (int e = 0; e < 4; ++e) {
            if (e & stride) continue;
            const int f = e | stride;
            const bool asc = ((4 * t + e) & size) == 0;
            const bool swap = asc ? nk_less(kl[f], kj[f], kl[e], kj[e]) : nk_less(kl[e], kj[e], kl[f], kj[f]);
            if (swap) { double tl = kl[e]; kl[e] = kl[f]; kl[f] = tl; int tj = kj[e]; kj[e] = kj[f]; kj[f] = tj; }
          }
        } else {
          const int m = stride >> 2;
          const bool keep_min = ((t & m) == 0) == (((4 * t) & size) == 0);
          if (stride < 256) {
            for (int e = 0; e < 4; ++e) {
              const double ol = __shfl_xor(kl[e], m, 64);
              const int ojv = __shfl_xor(kj[e], m, 64);
              sel(kl[e], kj[e], ol, ojv, keep_min);
            }
          } else {
            for (int e = 0; e < 4; ++e) { sl[4 * t + e] = kl[e]; sj[4 * t + e] = kj[e]; }
            __syncthreads();
            const int q = 4 * (t ^ m);
            double ol[4]; int ojv[4];
            for (int e = 0; e < 4; ++e) { ol[e] = sl[q + e]; ojv[e] = sj[q + e]; }
            __syncthreads();
            for (int e = 0; e < 4; ++e) sel(kl[e], kj[e], ol[e], ojv[e], keep_min);
          }
        }
      }
    }
  }
  for (int e = 0; e < 4; ++e) {
    const int p = 4 * t + e;
    if (p < k) { out[p] = kl[e]; oj[p] = kj[e]; }
  }
}

int main() {
  const int k = 4096, L = 4096;
  std::vector<double> h(k);
  unsigned s = 1;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = (double)(s >> 8) / 16777216.0; }
  double *din, *dout; int* dj;
  hipMalloc(&din, k * 8); hipMalloc(&dout, k * 8); hipMalloc(&dj, k * 4);
  hipMemcpy(din, h.data(), k * 8, hipMemcpyHostToDevice);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      for (int i = 0; i < 200; ++i) {
        if (mode == 0) hipLaunchKernelGGL(sort_k<0>, dim3(1), dim3(L / 4), 0, 0, din, dout, dj, k, L);
        else hipLaunchKernelGGL(sort_k<1>, dim3(1), dim3(L / 4), 0, 0, din, dout, dj, k, L);
      }
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("mode %d: %.2f us per launch\n", mode, ms * 1000 / 200);
    }
  }
  std::vector<double> o(k); hipMemcpy(o.data(), dout, k * 8, hipMemcpyDeviceToHost);
  bool sorted = true; for (int i = 1; i < k; ++i) sorted = sorted && o[i - 1] <= o[i];
  printf("sorted %d\n", (int)sorted);
  return 0;
}
