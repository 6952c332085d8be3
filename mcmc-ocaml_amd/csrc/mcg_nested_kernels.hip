// mcg_nested_kernels.hip -- order maintenance and bookkeeping kernels of the nested sampler.
//
// Keys (ll, tie, slot) are unique (tie is unique per point), so "ascending" is a strict total
// order and every sort / merge below has exactly one answer -- the same one the oracle's qsort
// and merge produce.  tie: initial points get their slot index, the m-th replacement gets -m,
// which reproduces the reference's tie order (stable initial sort, nested.ml:132; a new point is
// inserted before equal likelihoods, the strict > of nested.ml:36).
#include "mcg_nested_kernel.h"

namespace mcg {

__device__ __forceinline__ bool key_less(double la, long long ta, double lb, long long tb) {
  return la < lb || (la == lb && ta < tb);
}

// number of entries of the sorted run [lo, hi) strictly below key
__device__ __forceinline__ int64_t count_less(const double* ll, const long long* tie, int64_t lo,
                                              int64_t hi, double kl, long long kt) {
  int64_t a = lo, b = hi;
  while (a < b) {
    const int64_t m = (a + b) >> 1;
    if (key_less(ll[m], tie[m], kl, kt)) a = m + 1;
    else b = m;
  }
  return a - lo;
}

constexpr int kChunk = 2048;

// bitonic sort of independent 2048-key chunks in LDS
__global__ void __launch_bounds__(256) sort_chunks_kernel(double* ll, long long* tie, int* slot,
                                                          int64_t n, const NestDevState* stop) {
  if (stop && stop->stopped) return;
  __shared__ double sl[kChunk];
  __shared__ long long st[kChunk];
  __shared__ int ss[kChunk];
  const int64_t base = (int64_t)blockIdx.x * kChunk;
  for (int i = threadIdx.x; i < kChunk; i += blockDim.x) {
    const int64_t g = base + i;
    const bool ok = g < n;
    sl[i] = ok ? ll[g] : __builtin_inf();
    st[i] = ok ? tie[g] : 0x7FFFFFFFFFFFFFFFll;
    ss[i] = ok ? slot[g] : -1;
  }
  __syncthreads();
  for (int size = 2; size <= kChunk; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p = threadIdx.x; p < kChunk / 2; p += blockDim.x) {
        const int i = ((p & ~(stride - 1)) << 1) | (p & (stride - 1));   // stride is a power of 2
        const int j = i + stride;
        const bool up = (i & size) == 0;
        const bool gt = key_less(sl[j], st[j], sl[i], st[i]);
        if (gt == up) {
          const double tl = sl[i]; sl[i] = sl[j]; sl[j] = tl;
          const long long tt = st[i]; st[i] = st[j]; st[j] = tt;
          const int ts = ss[i]; ss[i] = ss[j]; ss[j] = ts;
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < kChunk; i += blockDim.x) {
    const int64_t g = base + i;
    if (g < n) {
      ll[g] = sl[i];
      tie[g] = st[i];
      slot[g] = ss[i];
    }
  }
}

// merge adjacent sorted runs of width w (rank scatter: each key finds its place in the partner)
__global__ void __launch_bounds__(256) merge_pass_kernel(const double* ll, const long long* tie,
                                                         const int* slot, double* oll, long long* otie,
                                                         int* oslot, int64_t n, int64_t w,
                                                         const NestDevState* stop) {
  if (stop && stop->stopped) return;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int64_t base = (e / (2 * w)) * (2 * w);
  const int64_t mid = base + w < n ? base + w : n;
  const int64_t end = base + 2 * w < n ? base + 2 * w : n;
  const double kl = ll[e];
  const long long kt = tie[e];
  int64_t pos;
  if (e < mid) pos = base + (e - base) + count_less(ll, tie, mid, end, kl, kt);
  else pos = base + (e - mid) + count_less(ll, tie, base, mid, kl, kt);
  oll[pos] = kl;
  otie[pos] = kt;
  oslot[pos] = slot[e];
}

hipError_t launch_sort_keys(double* ll, long long* tie, int* slot, double* tll, long long* ttie,
                            int* tslot, int64_t n, bool* result_in_tmp, hipStream_t s,
                            const NestDevState* stop) {
  const int64_t chunks = (n + kChunk - 1) / kChunk;
  hipLaunchKernelGGL(sort_chunks_kernel, dim3((unsigned)chunks), dim3(256), 0, s, ll, tie, slot, n, stop);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  bool in_tmp = false;
  for (int64_t w = kChunk; w < n; w <<= 1) {
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (!in_tmp)
      hipLaunchKernelGGL(merge_pass_kernel, dim3(grid), dim3(256), 0, s, ll, tie, slot, tll, ttie, tslot, n, w, stop);
    else
      hipLaunchKernelGGL(merge_pass_kernel, dim3(grid), dim3(256), 0, s, tll, ttie, tslot, ll, tie, slot, n, w, stop);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    in_tmp = !in_tmp;
  }
  *result_in_tmp = in_tmp;
  return hipSuccess;
}

// Sort this generation's k <= 4096 new keys in one workgroup (bitonic, 1024 threads, LDS).  The
// new keys' ties are -(mrep + j + 1), decreasing in j, so the key order is (ll ascending, j
// descending) and only (ll, j) enter LDS (48 KiB); tie and slot are rebuilt from j on the way out.
constexpr int kSmallSort = 4096;

__global__ void __launch_bounds__(1024) sort_new_small_kernel(const NestArgs a, double* oll,
                                                              long long* otie, int* oslot) {
  if (a.st->stopped) return;
  __shared__ double sl[kSmallSort];
  __shared__ int sj[kSmallSort];
  const int k = (int)a.k;
  int L = 2;
  while (L < k) L <<= 1;
  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    sl[i] = i < k ? a.newk_ll[i] : __builtin_inf();
    sj[i] = i < k ? i : -1;
  }
  __syncthreads();
  for (int size = 2; size <= L; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p = threadIdx.x; p < L / 2; p += blockDim.x) {
        const int i = ((p & ~(stride - 1)) << 1) | (p & (stride - 1));   // stride is a power of 2
        const int j = i + stride;
        const bool up = (i & size) == 0;
        const double li = sl[i], lj = sl[j];
        const int ji = sj[i], jj = sj[j];
        const bool j_less = lj < li || (lj == li && jj > ji);      // key j < key i
        if (j_less == up) {
          sl[i] = lj; sl[j] = li;
          sj[i] = jj; sj[j] = ji;
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    const int j = sj[i];
    oll[i] = sl[i];
    otie[i] = -(long long)(a.mrep + j + 1);
    oslot[i] = a.newk_slot[j];
  }
}

hipError_t launch_sort_new_small(const NestArgs& a, double* oll, long long* otie, int* oslot, hipStream_t s) {
  if (a.k > kSmallSort) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sort_new_small_kernel, dim3(1), dim3(1024), 0, s, a, oll, otie, oslot);
  return hipGetLastError();
}

// survivors keys[k..n) + k sorted new keys -> out[0..n)
__global__ void __launch_bounds__(256) merge_new_kernel(const NestArgs a, double* oll,
                                                        long long* otie, int* oslot,
                                                        const double* nl, const long long* nt,
                                                        const int* ns) {
  if (a.st->stopped) return;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = a.n, k = a.k, ns_ = n - k;
  if (e >= n) return;
  double kl;
  long long kt;
  int ks;
  int64_t pos;
  if (e < ns_) {
    kl = a.key_ll[k + e];
    kt = a.key_tie[k + e];
    ks = a.key_slot[k + e];
    pos = e + count_less(nl, nt, 0, k, kl, kt);
  } else {
    const int64_t b = e - ns_;
    kl = nl[b];
    kt = nt[b];
    ks = ns[b];
    pos = b + count_less(a.key_ll + k, a.key_tie + k, 0, ns_, kl, kt);
  }
  oll[pos] = kl;
  otie[pos] = kt;
  oslot[pos] = ks;
}

hipError_t launch_merge_new(const NestArgs& a, double* out_ll, long long* out_tie, int* out_slot,
                            const double* new_ll, const long long* new_tie, const int* new_slot,
                            hipStream_t s) {
  const unsigned grid = (unsigned)((a.n + 255) / 256);
  hipLaunchKernelGGL(merge_new_kernel, dim3(grid), dim3(256), 0, s, a, out_ll, out_tie, out_slot,
                     new_ll, new_tie, new_slot);
  return hipGetLastError();
}

// retire the k lowest (replace_live_point, nested.ml:26-43, slot form): copy each retired row to
// the dead buffer, put walker j's point into the freed slot, emit its key and ll + log dv
__global__ void __launch_bounds__(256) retire_kernel(const NestArgs a, int D) {
  if (a.st->stopped) return;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.k) return;
  const int s = a.key_slot[j];
  const int64_t m = a.mrep + j;
  for (int d = 0; d < D; ++d) a.dead_x[m * D + d] = a.x[(int64_t)s * D + d];
  const double lls = a.ll[s];
  a.dead_ll[m] = lls;
  a.dead_lp[m] = a.lp[s];
  const double lv = a.st->log_vol + a.prefix[j];
  a.tv[j] = lls + (lv + a.qadd[j]);                 // nested.ml:138-141 (log_dv incl. :140)
  for (int d = 0; d < D; ++d) a.x[(int64_t)s * D + d] = a.nx[j * D + d];
  a.ll[s] = a.nll[j];
  a.lp[s] = a.nlp[j];
  a.newk_ll[j] = a.nll[j];
  a.newk_tie[j] = -(long long)(m + 1);
  a.newk_slot[j] = s;
}

hipError_t launch_retire(const NestArgs& a, int D, hipStream_t s) {
  const unsigned grid = (unsigned)((a.k + 255) / 256);
  hipLaunchKernelGGL(retire_kernel, dim3(grid), dim3(256), 0, s, a, D);
  return hipGetLastError();
}

// est = lse(est, tree_lse(tv)) with a fixed pairwise tree; log_vol += sum_j log1p(-1/(n-j))
__global__ void __launch_bounds__(1024) estimate_kernel(const NestArgs a) {
  if (a.st->stopped) return;
  double* v = a.tv;
  const int64_t p2 = a.tv_len;
  for (int64_t i = a.k + threadIdx.x; i < p2; i += blockDim.x) v[i] = -__builtin_inf();
  __syncthreads();
  for (int64_t s = p2 >> 1; s >= 1; s >>= 1) {
    for (int64_t i = threadIdx.x; i < s; i += blockDim.x) v[i] = plse(v[i], v[i + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.st->est = plse(a.st->est, v[0]);
    a.st->log_vol = a.st->log_vol + a.prefix[a.k];
  }
}

hipError_t launch_estimate(const NestArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(estimate_kernel, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError();
}

// remaining_integral_negligable (nested.ml:45-48) on the replaced live set
__global__ void stop_kernel(const NestArgs a, const double* final_ll) {
  if (a.st->stopped) return;
  const double live = a.st->log_vol + final_ll[a.n - 1];
  if (live - plse(a.st->est, live) <= a.log_epsrel) a.st->stopped = 1;
  if (a.st->error) a.st->stopped = 1;
  a.st->gen_done += 1;
}

hipError_t launch_stop(const NestArgs& a, const double* final_ll, hipStream_t s) {
  hipLaunchKernelGGL(stop_kernel, dim3(1), dim3(1), 0, s, a, final_ll);
  return hipGetLastError();
}

}  // namespace mcg
