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

// Sort this generation's k <= 4096 new keys.  The new keys' ties are -(mrep + j + 1), decreasing
// in j, so the key order is (ll ascending, j descending) and only (ll, j) move; tie and slot are
// rebuilt from j at the end.  One workgroup would be bound by its CU's LDS unit (every exchange
// of a bitonic network goes through it), so the sort is spread over CUs:
//   1. sort_runs_kernel: ceil(k/256) single-wave workgroups each sort a run of 256 keys, lane l
//      holding positions 4l .. 4l+3: strides 1, 2 inside the lane, strides 4 .. 128 by
//      shuffles with lane l ^ (stride/4) -- no LDS storage, no barriers;
//   2. rank_merge_kernel: each key's final position = its index in its run + the number of keys
//      of every other run that precede it (binary searches; ties between runs broken by run
//      order, which only pads can need -- real keys are unique).
constexpr int kSmallSort = 4096;
constexpr int kRun = 256;

__device__ __forceinline__ bool nk_less(double la, int ja, double lb, int jb) {
  return la < lb || (la == lb && ja > jb);
}

__global__ void __launch_bounds__(64) sort_runs_kernel(const NestArgs a, double* rl, int* rj) {
  if (a.st->stopped) return;
  const int k = (int)a.k;
  const int t = threadIdx.x;
  const int base = blockIdx.x * kRun;
  double kl[4];
  int kj[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int p = base + 4 * t + e;
    kl[e] = p < k ? a.newk_ll[p] : __builtin_inf();
    kj[e] = p < k ? p : -1;
  }
#pragma unroll
  for (int size = 2; size <= kRun; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride <= 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (e & stride) continue;
          const int f = e | stride;
          const bool asc = ((4 * t + e) & size) == 0;
          const bool swap = asc ? nk_less(kl[f], kj[f], kl[e], kj[e]) : nk_less(kl[e], kj[e], kl[f], kj[f]);
          if (swap) {
            const double tl = kl[e]; kl[e] = kl[f]; kl[f] = tl;
            const int tj = kj[e]; kj[e] = kj[f]; kj[f] = tj;
          }
        }
      } else {
        const int m = stride >> 2;                       // partner lane t ^ m
        const bool keep_min = ((t & m) == 0) == (((4 * t) & size) == 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double ol = __shfl_xor(kl[e], m, 64);
          const int oj = __shfl_xor(kj[e], m, 64);
          if (nk_less(ol, oj, kl[e], kj[e]) == keep_min) {
            kl[e] = ol;
            kj[e] = oj;
          }
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    rl[base + 4 * t + e] = kl[e];
    rj[base + 4 * t + e] = kj[e];
  }
}

// All runs staged in LDS (<= 48 KiB), then every run's binary search advances in lockstep
// (one LDS read per run per round, eight rounds), so the reads of the other runs overlap.
__global__ void __launch_bounds__(256) rank_merge_kernel(const NestArgs a, const double* rl, const int* rj,
                                                         int nruns, double* oll, long long* otie, int* oslot) {
  if (a.st->stopped) return;
  __shared__ double sl[kSmallSort];
  __shared__ int sj[kSmallSort];
  const int n = nruns * kRun;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    sl[i] = rl[i];
    sj[i] = rj[i];
  }
  __syncthreads();
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const int r = g / kRun;
  const double l = sl[g];
  const int j = sj[g];
  if (j < 0) return;                                 // padding
  constexpr int kMaxRuns = kSmallSort / kRun;
  int lo[kMaxRuns];
#pragma unroll
  for (int q = 0; q < kMaxRuns; ++q) lo[q] = 0;
  // lo[q] = number of entries of run q before the key: strictly less for q > r, less or equal
  // (an equal key can only be padding) for q < r
#pragma unroll
  for (int w = kRun >> 1; w >= 1; w >>= 1) {
#pragma unroll
    for (int q = 0; q < kMaxRuns; ++q) {
      if (q >= nruns || q == r) continue;
      const int m = q * kRun + lo[q] + w - 1;
      const double ml = sl[m];
      const int mj = sj[m];
      const bool before = nk_less(ml, mj, l, j) || (q < r && ml == l && mj == j);
      if (before) lo[q] += w;
    }
  }
  int pos = g - r * kRun;
#pragma unroll
  for (int q = 0; q < kMaxRuns; ++q) {
    if (q >= nruns || q == r) continue;
    // the last probe of the halving search: the entry at lo[q] itself
    const int m = q * kRun + lo[q];
    if (lo[q] < kRun) {
      const double ml = sl[m];
      const int mj = sj[m];
      if (nk_less(ml, mj, l, j) || (q < r && ml == l && mj == j)) lo[q] += 1;
    }
    pos += lo[q];
  }
  oll[pos] = l;
  otie[pos] = -(long long)(a.mrep + j + 1);
  oslot[pos] = a.newk_slot[j];
}

hipError_t launch_sort_new_small(const NestArgs& a, double* rl, int* rj, double* oll, long long* otie,
                                 int* oslot, hipStream_t s) {
  if (a.k > kSmallSort) return hipErrorInvalidValue;
  const int nruns = (int)((a.k + kRun - 1) / kRun);
  hipLaunchKernelGGL(sort_runs_kernel, dim3(nruns), dim3(64), 0, s, a, rl, rj);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(rank_merge_kernel, dim3((nruns * kRun + 255) / 256), dim3(256), 0, s, a, rl, rj, nruns,
                     oll, otie, oslot);
  return hipGetLastError();
}

__device__ __forceinline__ void stop_test(const NestArgs& a, double max_ll);

// survivors keys[k..n) + k sorted new keys -> out[0..n) by rank scatter; the thread placing the
// largest key also runs the stop test of the generation.  (A two-level search with LDS-staged
// samples measured slower: 29 vs 12 us at C3 -- the per-block sample loads cost more than the
// L2-resident binary searches they save.)
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
  if (pos == n - 1) stop_test(a, kl);
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
// the dead buffer, put walker j's point into the freed slot, emit its key and ll + log dv.
// One thread per (point, dim) element; the dim-0 thread also moves the point's scalars.
__global__ void __launch_bounds__(256) retire_kernel(const NestArgs a, int D) {
  if (a.st->stopped) return;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.k * D) return;
  const int64_t j = g / D;
  const int d = (int)(g - j * D);
  const int s = a.key_slot[j];
  const int64_t m = a.mrep + j;
  a.dead_x[m * D + d] = a.x[(int64_t)s * D + d];
  a.x[(int64_t)s * D + d] = a.nx[j * D + d];
  if (d != 0) return;
  const double lls = a.ll[s];
  a.dead_ll[m] = lls;
  a.dead_lp[m] = a.lp[s];
  const double lv = a.st->log_vol + a.prefix[j];
  a.tv[j] = lls + (lv + a.qadd[j]);                 // nested.ml:138-141 (log_dv incl. :140)
  a.ll[s] = a.nll[j];
  a.lp[s] = a.nlp[j];
  a.newk_ll[j] = a.nll[j];
  a.newk_tie[j] = -(long long)(m + 1);
  a.newk_slot[j] = s;
}

hipError_t launch_retire(const NestArgs& a, int D, hipStream_t s) {
  const unsigned grid = (unsigned)((a.k * D + 255) / 256);
  hipLaunchKernelGGL(retire_kernel, dim3(grid), dim3(256), 0, s, a, D);
  return hipGetLastError();
}

// est = lse(est, tree_lse(tv)) with a fixed pairwise tree; log_vol += sum_j log1p(-1/(n-j)).
// The tree runs in LDS when the padded generation fits (tv_len <= 4096), else in global memory.
constexpr int kEstLds = 4096;

__global__ void __launch_bounds__(1024) estimate_kernel(const NestArgs a) {
  if (a.st->stopped) return;
  __shared__ double sv[kEstLds];
  __shared__ double2 s_lt[kLogTabN];                 // log table staged in LDS (per-level gathers)
  for (int i = threadIdx.x; i < kLogTabN; i += blockDim.x) s_lt[i] = kLogTab[i];
  const int64_t p2 = a.tv_len;
  const bool lds = p2 <= kEstLds;
  double* v = lds ? sv : a.tv;
  for (int64_t i = threadIdx.x; i < p2; i += blockDim.x) {
    if (i >= a.k) v[i] = -__builtin_inf();
    else if (lds) v[i] = a.tv[i];
  }
  __syncthreads();
  for (int64_t s = p2 >> 1; s >= 1; s >>= 1) {
    for (int64_t i = threadIdx.x; i < s; i += blockDim.x) v[i] = plse(v[i], v[i + s], s_lt);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.st->est = plse(a.st->est, v[0], s_lt);
    a.st->log_vol = a.st->log_vol + a.prefix[a.k];
  }
}

hipError_t launch_estimate(const NestArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(estimate_kernel, dim3(1), dim3(1024), 0, s, a);
  return hipGetLastError();
}

// remaining_integral_negligable (nested.ml:45-48) on the replaced live set; run by the thread of
// merge_new_kernel that places the largest key (final_ll[n - 1])
__device__ __forceinline__ void stop_test(const NestArgs& a, double max_ll) {
  const double live = a.st->log_vol + max_ll;
  if (live - plse(a.st->est, live) <= a.log_epsrel) a.st->stopped = 1;
  if (a.st->error) a.st->stopped = 1;
  a.st->gen_done += 1;
}

}  // namespace mcg
