// mcg_nested_kernels.hip -- order maintenance and bookkeeping kernels of the nested sampler.
//
// Keys (ll, tie, slot) are unique (tie is unique per point), so "ascending" is a strict total
// order and every sort / merge below has exactly one answer -- the same one the oracle's qsort
// and merge produce.  tie: initial points get their slot index, the m-th replacement gets -m,
// which reproduces the reference's tie order (stable initial sort, nested.ml:132; a new point is
// inserted before equal likelihoods, the strict > of nested.ml:36).
#include <algorithm>
#include <cstdlib>

#include "mcg_nested_kernel.h"

namespace mcg {


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
  if (stop && nest_stopped(stop)) return;
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
  if (stop && nest_stopped(stop)) return;
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
// in j, so the key order is (ll ascending, j descending) and only (ll, j) decide it.  The keys
// are unique, so key j's position is its rank: the number of new keys below it.  The ranks are
// counted, not searched: block (A, B) of a (k/256) x (k/128) grid compares each key of run A with
// the 128 keys of sub-run B (LDS broadcast reads) and adds its count to rank[j] (integer atomics: the sum is
// order-independent and exact).  The last block to finish scatters every key to its rank.  One
// launch of 128 compares per lane replaces a run sort plus a rank merge, which were bound
// by their serial shuffle / search latencies (12 + 20 us per generation at k = 4096).
constexpr int kRun = 256;

// Last-workgroup hand-off (MI355X_MICROARCH.md, hand-offs with sc1 loads, first row): the
// handed-off bytes are stored sc1 (or are agent-scope atomics) and loaded sc1 (ld1 / st1 below),
// so no producer needs an L2 write-back (release); every wave waits for its stores, a workgroup
// barrier, then one lane counts.  The count is two-level (16 group counters, then a top counter
// added to by the workgroup completing its group): one counter taking every workgroup's add
// serialises them (measured: 6 us of spread over 512 workgroups).  The workgroup completing the
// top counter acquires once and runs the consumer part.  No workgroup waits on another.
__device__ __forceinline__ bool last_block_done(uint32_t* sync, uint32_t nblocks) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t nb = nblocks, g = blockIdx.x % kSyncGroups;
    const uint32_t gsize = (nb - g + kSyncGroups - 1) / kSyncGroups;
    const uint32_t ngroups = nb < (uint32_t)kSyncGroups ? nb : (uint32_t)kSyncGroups;
    uint32_t* gc = sync + (1 + g) * kSyncStride;
    int last = 0;
    if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
      __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1;
    }
    if (last) {
      // the consumer's one agent acquire (drops stale L1 / L2 copies of the handed-off lines)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

constexpr int kSub = 128;                            // keys of the compared-against sub-run

__global__ void __launch_bounds__(256) rank_count_kernel(const NestArgs a, int nruns, double* oll,
                                                         long long* otie, int* oslot) {
  NT_STAMP(2, 0);
  if (nest_stopped(a.st)) return;                         // grid-uniform: set by an earlier launch
  if (a.est_in_rank && blockIdx.x == gridDim.x - 1) {
    // the extra workgroup folds the generation into the running estimate (retire wrote tv),
    // beside the counting: off the generation's serial path
    __shared__ EstLds<kRun> el;
    estimate_body<kRun>(a, el);
    return;
  }
  const uint32_t ncount = gridDim.x - (a.est_in_rank ? 1u : 0u);
  // the retire kernel's slot writes (the walkers moved the dead rows and emitted the keys):
  // walker j's point into the slot it replaces, spread over the counting workgroups.  They run
  // after the counting and the hand-off (nothing in this kernel reads them; the next walk does,
  // after a kernel boundary), so their loads do not delay the count
  auto slot_writes = [&]() {
    if (!a.fuse_retire) return;
    const int64_t kD = a.k * a.row_bytes / 8, D = a.row_bytes / 8;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < kD; g += (int64_t)ncount * blockDim.x) {
      const int64_t j = g / D;
      const int64_t d = g - j * D;
      const int sj = a.newk_slot[j];
      a.x[(int64_t)sj * D + d] = a.nx[g];
      if (d == 0) {
        a.ll[sj] = a.nll[j];
        a.lp[sj] = a.nlp[j];
      }
    }
  };
  __shared__ double sl[kSub];
  __shared__ double s_ll[kSmallSort];                // last block: keys placed at their ranks
  __shared__ short s_j[kSmallSort];
  const int k = (int)a.k;
  const int A = (int)(blockIdx.x % nruns), B = (int)(blockIdx.x / nruns);
  const int t = threadIdx.x;
  const int b0 = B * kSub;
  const int nb = min(kSub, k - b0);
  if (t < nb) sl[t] = a.newk_ll[b0 + t];
  __syncthreads();
  NT_STAMP(2, 1);
  const int p = A * kRun + t;
  if (p < k) {
    const double l = a.newk_ll[p];
    int cnt = 0;
    if (nb == kSub) {
#pragma unroll 16
      for (int q = 0; q < kSub; ++q) {
        const double o = sl[q];
        cnt += (int)((o < l) | ((o == l) & (b0 + q > p)));   // nk order: ll asc, j desc
      }
    } else {
      for (int q = 0; q < nb; ++q) {
        const double o = sl[q];
        cnt += (int)((o < l) | ((o == l) & (b0 + q > p)));
      }
    }
    NT_STAMP(2, 2);
    if (cnt) atomicAdd(&a.rank[p], cnt);
  }
  const bool last = last_block_done(a.sync + kSyncUse, ncount);
  NT_STAMP(2, 3);
  if (!last) {
    slot_writes();
    return;
  }
  // the last block places every key at its rank in LDS (a random scatter from one CU is bound by
  // its store rate), then writes the sorted keys out coalesced
  constexpr int kPer = kSmallSort / kRun;
  int rr[kPer];
  double rl[kPer];
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int q = min(e * kRun + t, k - 1);
    rr[e] = ld1(a.rank + q);
    rl[e] = a.newk_ll[q];
  }
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int q = e * kRun + t;
    if (q < k) {
      s_ll[rr[e]] = rl[e];
      s_j[rr[e]] = (short)q;
    }
  }
  __syncthreads();
  NT_STAMP(2, 4);
  int js[kPer], sl_[kPer];
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int r = min(e * kRun + t, k - 1);
    js[e] = s_j[r];
    sl_[e] = a.newk_slot[js[e]];
  }
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int r = e * kRun + t;
    if (r < k) {
      oll[r] = s_ll[r];
      otie[r] = -(long long)(a.mrep + js[e] + 1);
      oslot[r] = sl_[e];
    }
  }
  NT_STAMP(2, 5);
  slot_writes();
}

hipError_t launch_sort_new_small(const NestArgs& a, double* oll, long long* otie, int* oslot,
                                 hipStream_t s) {
  if (a.k > kSmallSort || a.k < 1) return hipErrorInvalidValue;
  const int nruns = (int)((a.k + kRun - 1) / kRun), nsub = (int)((a.k + kSub - 1) / kSub);
  hipLaunchKernelGGL(rank_count_kernel, dim3((unsigned)(nruns * nsub + (a.est_in_rank ? 1 : 0))), dim3(kRun), 0, s,
                     a, nruns, oll, otie, oslot);
  return hipGetLastError();
}

// Search samples of a sorted key array staged in LDS: every S-th key (indices S-1, 2S-1, ...), at
// most `cap` of them; S is the smallest power of two >= 16 that keeps the count within cap.
struct KeySample {
  int64_t S;
  int n;
};
__device__ __forceinline__ KeySample key_sample(int64_t len, int cap, int64_t smin = 16) {
  int64_t S = smin;
  while (len / S > cap) S <<= 1;
  return KeySample{S, (int)(len / S)};
}

// count of the sorted keys [0, len) strictly below (kl, kt): the first levels in the LDS sample,
// the last log2 S in global memory
__device__ __forceinline__ int64_t count_less_2l(const double* ll, const long long* tie, int64_t len,
                                                 KeySample ks, const double* sll, const long long* stie,
                                                 double kl, long long kt) {
  int a = 0, b = ks.n;
  while (a < b) {
    const int m = (a + b) >> 1;
    if (key_less(sll[m], stie[m], kl, kt)) a = m + 1;
    else b = m;
  }
  const int64_t lo = (int64_t)a * ks.S;
  const int64_t hi = a < ks.n ? lo + ks.S - 1 : len;   // sample a is not below the key
  return lo + count_less(ll, tie, lo, hi, kl, kt);
}

// the new keys' sample: every 4th key (k <= 4096), so a survivor's search ends with two
// dependent global probes instead of four
constexpr int kSampNew = 1024, kSampSurv = 2048;
constexpr int64_t kSampNewMin = kSampNew >= 1024 ? 4 : 16;

// survivors keys[k..n) + k sorted new keys -> out[0..n) by rank scatter; the thread placing the
// largest key also counts the generation (the stop test runs at the start of the next walk).  Each binary search starts in an LDS
// sample of the array it searches (survivors search the new keys, new keys the survivors), so
// only its last log2 S probes are dependent global loads.
__global__ void __launch_bounds__(256) merge_new_kernel(const NestArgs a, double* oll,
                                                        long long* otie, int* oslot,
                                                        const double* nl, const long long* nt,
                                                        const int* ns) {
  NT_STAMP(3, 0);
  __shared__ double s_nl[kSampNew], s_sl[kSampSurv];
  __shared__ long long s_nt[kSampNew], s_st[kSampSurv];
  const int64_t n = a.n, k = a.k, ns_ = n - k;
  const int64_t e0 = (int64_t)blockIdx.x * blockDim.x, e = e0 + threadIdx.x;
  const bool has_surv = e0 < ns_, has_new = e0 + blockDim.x > ns_;   // block-uniform
  const double* sll = a.key_ll + k;
  const long long* stie = a.key_tie + k;
  const KeySample kn = key_sample(k, kSampNew, kSampNewMin), kv = key_sample(ns_, kSampSurv);
  KeySample kv_use = kv;
  // own key and the samples: all loads issued before the stop flag is read
  const int64_t ec = e < n ? e : n - 1;
  double kl;
  long long kt;
  int ks;
  if (ec < ns_) {
    kl = sll[ec];
    kt = stie[ec];
    ks = a.key_slot[k + ec];
  } else {
    kl = nl[ec - ns_];
    kt = nt[ec - ns_];
    ks = ns[ec - ns_];
  }
  if (has_surv) {
#pragma unroll
    for (int r = 0; r < (kSampNew + 255) / 256; ++r) {
      const int i = r * 256 + (int)threadIdx.x;
      if (i < kn.n) {
        const int64_t q = (int64_t)(i + 1) * kn.S - 1;
        s_nl[i] = nl[q];
        s_nt[i] = nt[q];
      }
    }
  }
  if (has_new) {
    // survivors' sample: from the compact sample the previous merge kept beside the keys
    // (contiguous loads) when k is a multiple of its spacing, else strided from the keys
    const bool compact = k % kKeySample == 0;
    int64_t m = 1;
    if (compact)
      while (ns_ / (kKeySample * m) > kSampSurv) m <<= 1;
    const KeySample kc{kKeySample * m, (int)(ns_ / (kKeySample * m))};
    const KeySample ku = compact ? kc : kv;
    constexpr int kPer = kSampSurv / 256;
    double tl[kPer];
    long long tt[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int i = min(r * 256 + (int)threadIdx.x, max(ku.n - 1, 0));
      if (compact) {
        const int64_t c = k / kKeySample + (int64_t)(i + 1) * m - 1;
        tl[r] = ku.n > 0 ? a.key_samp_ll[c] : 0.0;
        tt[r] = ku.n > 0 ? a.key_samp_tie[c] : 0;
      } else {
        const int64_t q = (int64_t)(i + 1) * ku.S - 1;
        tl[r] = ku.n > 0 ? sll[q] : 0.0;
        tt[r] = ku.n > 0 ? stie[q] : 0;
      }
    }
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int i = r * 256 + threadIdx.x;
      if (i < ku.n) {
        s_sl[i] = tl[r];
        s_st[i] = tt[r];
      }
    }
    kv_use = ku;
  }
  __syncthreads();
  if (nest_stopped(a.st)) return;
  NT_STAMP(3, 1);
  if (e >= n) return;
  int64_t pos;
  if (e < ns_) pos = e + count_less_2l(nl, nt, k, kn, s_nl, s_nt, kl, kt);
  else pos = (e - ns_) + count_less_2l(sll, stie, ns_, kv_use, s_sl, s_st, kl, kt);
  NT_STAMP(3, 2);
  oll[pos] = kl;
  otie[pos] = kt;
  oslot[pos] = ks;
  if (pos % kKeySample == kKeySample - 1) {          // the next generation's key sample
    a.out_samp_ll[pos / kKeySample] = kl;
    a.out_samp_tie[pos / kKeySample] = kt;
  }
  if (pos == n - 1) {
    a.st->max_ll = kl;
    __hip_atomic_fetch_add(&a.st->gen_done, 1LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  NT_STAMP(3, 3);
}

// merge_fused_block (mcg_nested_merge.h) as a kernel of its own, after the walk's boundary: its
// loads of the walkers' outputs are plain ones
template <int BS, int KCAP>
__global__ void __launch_bounds__(BS) merge_fused_kernel(const NestArgs a, double* oll, long long* otie,
                                                         int* oslot) {
  NT_STAMP(3, 0);
  if (nest_stopped(a.st)) return;                         // grid-uniform: set by an earlier launch
  const int nblk = (int)((a.n - a.k + BS - 1) / BS);
  if ((int)blockIdx.x == nblk) {                          // the running estimate (retire wrote tv)
    __shared__ EstLds<BS> el;
    estimate_body<BS>(a, el);
    return;
  }
  __shared__ MergeLds<BS, KCAP> ml;
  merge_fused_block<BS, KCAP, false>(a, oll, otie, oslot, (int)blockIdx.x, ml);
}

hipError_t launch_merge_fused(const NestArgs& a, double* oll, long long* otie, int* oslot, hipStream_t s) {
  if (a.k > kFusedMax || a.k < 1 || !a.est_in_rank) return hipErrorInvalidValue;
  // k <= 4096: 512 survivors a workgroup by default.  Every workgroup classifies all k new keys
  // (f64 / i64 compares, the launch's bulk), so halving the workgroups halves that work; 256 a
  // workgroup (MCG_MERGE_BS=256, the round-4 shape) classifies twice as much in total
  static const int merge_bs = [] {
    const char* e = getenv("MCG_MERGE_BS");
    return e && atoi(e) == 256 ? 256 : 512;
  }();
  if (a.k <= kSmallSort && merge_bs == 256) {
    const unsigned nblk = (unsigned)((a.n - a.k + 255) / 256);
    hipLaunchKernelGGL((merge_fused_kernel<256, kSmallSort>), dim3(nblk + 1), dim3(256), 0, s, a, oll, otie, oslot);
  } else if (a.k <= kSmallSort) {
    const unsigned nblk = (unsigned)((a.n - a.k + 511) / 512);
    hipLaunchKernelGGL((merge_fused_kernel<512, kSmallSort>), dim3(nblk + 1), dim3(512), 0, s, a, oll, otie, oslot);
  } else {
    const unsigned nblk = (unsigned)((a.n - a.k + 511) / 512);
    hipLaunchKernelGGL((merge_fused_kernel<512, kFusedMax>), dim3(nblk + 1), dim3(512), 0, s, a, oll, otie, oslot);
  }
  return hipGetLastError();
}

// Split merge, head (mcg_nested_merge.h): workgroups [0, nb) are the merge's first survivor
// blocks (512 survivors each, positions < k), workgroup nb folds L_max and the generation count
// (the estimate was folded during the walk, nest_est_role), workgroups past it put the new points into the slots they replace (the
// next walk reads them).  The tail (positions >= k) runs in the next walk's launch
// (nest_tail_block) or, after the last generation, in merge_tail_kernel.
__global__ void __launch_bounds__(kHeadT) merge_head_kernel(const NestArgs a, double* oll, long long* otie,
                                                            int* oslot, int nb) {
  NT_STAMP(3, 0);
  if (nest_stopped(a.st)) return;                         // grid-uniform: set by an earlier launch
  __shared__ union HeadU {
    MergeLds<kHeadT, kSmallSort> m;
    EstLds<kHeadT> e;
  } lds;
  const int b = (int)blockIdx.x;
  if (b < nb) {
    NestArgs h = a;
    h.fuse_retire = 0;
    merge_fused_block<kHeadT, kSmallSort, false, MergeNoWait, kMergeHead>(h, oll, otie, oslot, b, lds.m);
  } else if (b == nb) {
    // (the estimate was folded during the walk: nest_est_role)
    head_lmax(a, head_lmax_load(a), lds.e.sv);
    NT_STAMP(1, 4);
  } else {
    const int64_t D = a.row_bytes / 8, kD = a.k * D;
    const int64_t stride = (int64_t)(gridDim.x - nb - 1) * kHeadT;
    for (int64_t g = (int64_t)(b - nb - 1) * kHeadT + threadIdx.x; g < kD; g += stride) {
      const int64_t j = g / D;
      const int64_t d = g - j * D;
      const int sj = a.newk_slot[j];
      a.x[(int64_t)sj * D + d] = a.nx[g];
      if (d == 0) {
        a.ll[sj] = a.nll[j];
        a.lp[sj] = a.nlp[j];
      }
    }
  }
}

hipError_t launch_merge_head(const NestArgs& a, double* oll, long long* otie, int* oslot, hipStream_t s) {
  if (a.k > kSmallSort || a.k < 1 || !a.est_in_rank || a.tv_len > kEstPer * kHeadT) return hipErrorInvalidValue;
  const int64_t ns = a.n - a.k;
  const int nb = (int)std::min<int64_t>((a.k + kHeadT - 1) / kHeadT, (ns + kHeadT - 1) / kHeadT);
  const int64_t kD = a.k * (a.row_bytes / 8);
  const unsigned nsw = (unsigned)std::max<int64_t>(1, std::min<int64_t>((kD + kHeadT - 1) / kHeadT, 256));
  hipLaunchKernelGGL(merge_head_kernel, dim3(nb + 1 + nsw), dim3(kHeadT), 0, s, a, oll, otie, oslot, nb);
  return hipGetLastError();
}

// the tail of the last generation's merge when no walk ran it (the run ended at max_dead)
__global__ void __launch_bounds__(256) merge_tail_kernel(const NestArgs a) {
  nest_tail_block(a, (int)blockIdx.x);
}

hipError_t launch_merge_tail(const NestArgs& a, hipStream_t s) {
  if (a.tl_nblk <= 0) return hipSuccess;
  hipLaunchKernelGGL(merge_tail_kernel, dim3((unsigned)a.tl_nblk), dim3(256), 0, s, a);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) key_sample_kernel(const double* ll, const long long* tie,
                                                         int64_t n, double* sll, long long* stie,
                                                         NestDevState* st) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && st) st->max_ll = ll[n - 1];          // the initial live set's L_max
  if (c >= n / kKeySample) return;
  sll[c] = ll[(c + 1) * kKeySample - 1];
  stie[c] = tie[(c + 1) * kKeySample - 1];
}

hipError_t launch_key_sample(const double* ll, const long long* tie, int64_t n, double* sll,
                             long long* stie, hipStream_t s, NestDevState* st) {
  const int64_t ns = n / kKeySample;
  hipLaunchKernelGGL(key_sample_kernel, dim3((unsigned)(ns / 256 + 1)), dim3(256), 0, s, ll, tie, n, sll, stie, st);
  return hipGetLastError();
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
// One thread per (point, dim) element; the dim-0 thread also moves the point's scalars.  The last
// workgroup to finish folds the generation into the running estimate (estimate_body).
__global__ void __launch_bounds__(kRetireBlock) retire_kernel(const NestArgs a, int D) {
  NT_STAMP(1, 0);
  if (nest_stopped(a.st)) return;                         // grid-uniform: set by an earlier launch
  NT_STAMP(1, 1);
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < a.k * D) {
    const int64_t j = g / D;
    const int d = (int)(g - j * D);
    const int s = a.key_slot[j];
    const int64_t m = a.mrep + j;
    a.dead_x[m * D + d] = a.x[(int64_t)s * D + d];
    a.x[(int64_t)s * D + d] = a.nx[j * D + d];
    if (d == 0) {
      const double lls = a.ll[s];
      put_dead(a, m, lls, a.lp[s]);
      const double lv = a.st->log_vol[gen_par(a)] + a.prefix[j];
      st1(a.tv + j, lls + (lv + a.qadd[j]));        // nested.ml:138-141 (log_dv incl. :140)
      a.ll[s] = a.nll[j];
      a.lp[s] = a.nlp[j];
      a.newk_ll[j] = a.nll[j];
      a.newk_tie[j] = -(long long)(m + 1);
      a.newk_slot[j] = s;
      if (a.rank) a.rank[j] = 0;
    }
  }
  if (a.est_in_rank) return;                         // rank_count_kernel folds the estimate
  NT_STAMP(1, 2);
  const bool last = last_block_done(a.sync, gridDim.x);
  NT_STAMP(1, 3);
  if (!last) return;
  __shared__ EstLds<kRetireBlock> el;
  estimate_body<kRetireBlock>(a, el);
  NT_STAMP(1, 4);
}

hipError_t launch_retire(const NestArgs& a, int D, hipStream_t s) {
  const unsigned grid = (unsigned)((a.k * D + kRetireBlock - 1) / kRetireBlock);
  hipLaunchKernelGGL(retire_kernel, dim3(grid), dim3(kRetireBlock), 0, s, a, D);
  return hipGetLastError();
}



// diagnostics (MCG_NESTED_CHECK): records in out[0..1] the first generation (+1) whose keys
// [0, n) are not strictly ascending in (ll, tie), out[2] the count of such pairs
__global__ void __launch_bounds__(256) check_sorted_kernel(const double* ll, const long long* tie,
                                                           int64_t n, long long gen, long long* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i + 1 >= n) return;
  if (!key_less(ll[i], tie[i], ll[i + 1], tie[i + 1])) {
    atomicCAS((unsigned long long*)out, 0ull, (unsigned long long)(gen + 1));
    atomicAdd((unsigned long long*)(out + 2), 1ull);
  }
}

hipError_t launch_check_sorted(const double* ll, const long long* tie, int64_t n, long long gen,
                               long long* out, hipStream_t s) {
  if (n < 2) return hipSuccess;
  hipLaunchKernelGGL(check_sorted_kernel, dim3((unsigned)((n + 254) / 256)), dim3(256), 0, s, ll, tie, n, gen, out);
  return hipGetLastError();
}


// the final live rows in key order (slot[j] of the sorted keys), written behind the dead rows
__global__ void __launch_bounds__(256) gather_live_kernel(const double* x, const double* ll, const double* lp,
                                                          const int* slot, int64_t n, int D, double* ox,
                                                          double* oll, double* olp) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n * D) return;
  const int64_t j = g / D;
  const int d = (int)(g - j * D);
  const int s = slot[j];
  ox[g] = x[(int64_t)s * D + d];
  if (d == 0) {
    oll[j] = ll[s];
    olp[j] = lp[s];
  }
}

hipError_t launch_gather_live(const double* x, const double* ll, const double* lp, const int* slot, int64_t n,
                              int D, double* ox, double* oll, double* olp, hipStream_t s) {
  hipLaunchKernelGGL(gather_live_kernel, dim3((unsigned)((n * D + 255) / 256)), dim3(256), 0, s, x, ll, lp, slot,
                     n, D, ox, oll, olp);
  return hipGetLastError();
}


// the run's output rows for a device-side exchange (mcg_nested_rows_into): element e of the
// [n][ncol] block, ncol = (D if points) + 2; row r = (x[r][0..D) | ll[r], lp[r])
__global__ void __launch_bounds__(256) nested_rows_kernel(const double* __restrict__ x, int Dk, int D,
                                                          const double* __restrict__ ll,
                                                          const double* __restrict__ lp, int64_t n,
                                                          double* __restrict__ out, int64_t stride, int pts) {
  const int ncol = (pts ? D : 0) + 2;
  const int64_t tot = n * ncol;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / ncol;
    const int c = (int)(e - r * ncol);
    const int cd = pts ? D : 0;
    out[r * stride + c] = c < cd ? x[r * Dk + c] : c == cd ? ll[r] : lp[r];
  }
}

hipError_t launch_nested_rows(const double* x, int Dk, int D, const double* ll, const double* lp, int64_t n,
                              double* out, int64_t stride, int pts, hipStream_t s) {
  const int64_t tot = n * ((pts ? D : 0) + 2);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((tot + 255) / 256, 16384));
  hipLaunchKernelGGL(nested_rows_kernel, dim3(grid), dim3(256), 0, s, x, Dk, D, ll, lp, n, out, stride, pts);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) walk_draws_kernel(const NestArgs a, int64_t mrep) {
  walk_draws_fill(a, mrep, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x, kLogTab);
}

hipError_t launch_walk_draws(const NestArgs& a, int64_t mrep, hipStream_t s) {
  if (!a.rt_ix) return hipSuccess;
  const int64_t tot = a.k * a.nmcmc;
  const unsigned grid = (unsigned)std::min<int64_t>((tot + 255) / 256, 4096);
  hipLaunchKernelGGL(walk_draws_kernel, dim3(grid), dim3(256), 0, s, a, mrep);
  return hipGetLastError();
}

}  // namespace mcg
