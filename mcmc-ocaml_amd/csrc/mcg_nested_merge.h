// mcg_nested_merge.h -- the estimate fold and the one-launch key merge of a nested generation
// (DESIGN.md §5.3), as device functions: run as kernels of their own (mcg_nested_kernels.hip) or
// as the merge role of the walk kernel (nest_walk_kernel<..., FM>, mcg_nested_kernel.h), which
// then hands the walkers' outputs off inside the launch.  Included by mcg_nested_kernel.h, after
// NestArgs, NT_STAMP and wt_store, inside namespace mcg.
#pragma once

__device__ __forceinline__ bool key_less(double la, long long ta, double lb, long long tb) {
  return (la < lb) | ((la == lb) & (ta < tb));       // branchless: both halves are cheap
}


constexpr int kSmallSort = 4096;                     // the largest k of the one-launch sorts

template <typename T>
__device__ __forceinline__ T ld1(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// est = lse(est, G) and log_vol += sum_j log1p(-1/(n-j)), where G is the log-sum of this
// generation's terms tv[0..k): tv[0] for k = 1 (the reference's fold, nested.ml:138-141), else
// M + log(sum exp(tv_j - M)) with M = max tv and the exps added by a fixed pairwise tree (pad to a
// power of two with 0; i + s into i) -- the oracle's tree_lse, operation for operation.  Run by
// the last workgroup of the retire kernel (1024 threads: up to 16,384 retirements) or by an extra
// rank-count workgroup (256 threads: k <= 4096), after every tv[j] is stored.
constexpr int kEstPer = 16;                          // retirements per thread of the estimate
constexpr int kRetireBlock = 1024;

// the estimate's LDS (a struct, so a kernel can overlay it with other roles' LDS)
template <int B>
struct EstLds {
  double sv[B];
  double s_max[B / 64];
  double2 s_lt[kLogTabN];                            // log table staged in LDS
};

template <int B>   // workgroup size; generations up to kEstPer * B retirements
__device__ __forceinline__ void estimate_body(const NestArgs& a, EstLds<B>& L) {
  double* const sv = L.sv;
  double* const s_max = L.s_max;
  double2* const s_lt = L.s_lt;
  for (int i = threadIdx.x; i < kLogTabN; i += B) s_lt[i] = kLogTab[i];
  const int64_t k = a.k, p2 = a.tv_len;              // p2 <= kEstPer * B (checked on the host)
  const int t = threadIdx.x;
  // thread t holds v[t + B q]: all loads in flight together (tv was stored sc1 by the retire
  // workgroups)
  double e[kEstPer];
  double m = -__builtin_inf();
#pragma unroll
  for (int q = 0; q < kEstPer; ++q) {
    const int64_t i = (int64_t)q * B + t;
    e[q] = ld1(a.tv + (i < k ? i : k - 1));
  }
#pragma unroll
  for (int q = 0; q < kEstPer; ++q)
    if ((int64_t)q * B + t < k) m = fmax(m, e[q]);
  NT_STAMP(1, 5);
  // M: the block max (exact in any order)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  if ((t & 63) == 0) s_max[t >> 6] = m;
  __syncthreads();
  double M = s_max[0];
#pragma unroll
  for (int w = 1; w < B / 64; ++w) M = fmax(M, s_max[w]);
  NT_STAMP(1, 6);
  const double v_first = e[0];                       // tv[0] (t == 0): the k == 1 fold
  double x = 0.0;
  if (k > 1 && M != -__builtin_inf()) {
    // the same tree (v[i] += v[i + s], s = p2/2 .. 1) with its levels where the data are:
    // s >= B pairs elements of one thread (i and i + s are both t mod B), in its registers;
    // 512 .. 64 in LDS after one barrier; 32 .. 1 by shuffles inside wave 0
    // (rows q B .. q B + B - 1 past k skip their exps: a uniform branch; the k = 4096 estimate of
    // a 1024-thread workgroup evaluated 16 exps a thread for 4 it needed)
#pragma unroll
    for (int q = 0; q < kEstPer; ++q) {
      if ((int64_t)q * B < k) e[q] = ((int64_t)q * B + t < k) ? pexp(e[q] - M) : 0.0;
      else e[q] = 0.0;
    }
    int64_t s = p2 >> 1;
    for (; s >= B; s >>= 1) {
      const int d = (int)(s / B);
#pragma unroll
      for (int q = 0; q < kEstPer / 2; ++q)
        if (q < d) e[q] = e[q] + e[q + d];
    }
    x = e[0];
    if (s >= 64) {
      // levels s = 512 .. 64 after one barrier: final v[i] (i < 64) combines v[i + 64 m],
      // m < 2s/64, by the same tree (m with m + d, d = s/64 .. 1) in wave 0's registers
      sv[t] = x;
      __syncthreads();
      if (t < 64) {
        const int nm = (int)(2 * s / 64);
        double g[B / 64];
#pragma unroll
        for (int q = 0; q < B / 64; ++q) g[q] = q < nm ? sv[t + 64 * q] : 0.0;
#pragma unroll
        for (int d = B / 128; d >= 1; d >>= 1)
          if (d < nm)
#pragma unroll
            for (int q = 0; q < d; ++q) g[q] = g[q] + g[q + d];
        x = g[0];
      }
      s = 32;
    }
    for (; s >= 1; s >>= 1) x = x + __shfl_down(x, (unsigned)s, 64);
  }
  NT_STAMP(1, 7);
  if (t == 0) {
    const double G = k == 1 ? v_first : (M == -__builtin_inf() ? M : M + plog(x, s_lt));
    const int g0 = gen_par(a), g1 = g0 ^ 1;
    a.st->est[g1] = plse(a.st->est[g0], G, s_lt);
    a.st->log_vol[g1] = a.st->log_vol[g0] + a.prefix[k];
  }
}

// One-kernel sort + merge of a generation's k <= 4096 unsorted new keys into the n - k survivors
// (DESIGN.md §5.3, round 3).  Survivor block b (BS = 256 consecutive survivors s[256b, 256b + 256))
// owns the key range [s[256b], s[256b + 256]) (block 0 from -inf, the last block to +inf), so
// every new key belongs to exactly one block.  Each block loads the k new ll into registers (a
// new key's tie, -(mrep + j + 1), is known from its index j), classifies them as they land (wave
// ballots), and finds
//   c_lo = #new keys below its range          (every new key below s[256b]),
//   its subset: the new keys inside its range, ranked among themselves by counting;
// then survivor i goes to  i + c_lo + #subset below it,  and subset key x to
//   256b + #block survivors below x + c_lo + rank of x in the subset.
// No sorted new-key array, no hand-off between workgroups: the old rank count -> merge pair
// (two launches, 11.5 + 11.1 us at C3) becomes one launch.  An extra workgroup folds the running
// estimate; every merge workgroup then takes a share of the new points' slot writes.
constexpr int kFusedMax = 2 * kSmallSort;                // the largest k of the one-launch merge

// BS: workgroup size = survivors per workgroup; KCAP: the largest k (new keys per thread
// KCAP / BS, the block's subset staged in LDS up to KCAP keys).  k <= 4096: <256, 4096>; up to
// 8192: <512, 8192> (98 KB of LDS, one workgroup per CU: 512 survivors a workgroup keep the
// grid to one round on the 256 CUs)
template <int BS, int KCAP>
struct MergeLds {
  double s_sv_l[BS];                                      // this block's survivors
  long long s_sv_t[BS];
  double s_subl[KCAP];                                    // subset: new ll and walker index j,
  short s_sub[KCAP];                                      // in gather order
  short s_srt[KCAP];                                      // subset positions in key order
  int s_subslot[KCAP];                                    // subset slots (loaded with the ll)
  int s_scan[2 * (BS / 64)];
};

// Block b of the merge.  SC1: the walkers' outputs (new keys, points, ll, lp) were handed off
// inside the same launch (nest_walk_kernel's merge role), so they are loaded sc1 (ld1); after a
// kernel boundary plain loads.  wait(): called by every thread once the survivors' loads (the
// previous generation's keys) are in flight and before any load of the walkers' outputs; false
// (uniform) ends the block.
struct MergeNoWait {
  __device__ bool operator()() const { return true; }
};

// PART (split merge): kMergeAll stores every position; kMergeHead only
// positions < k (the head kernel, whose other workgroups fold the estimate, L_max and the
// generation count and write the new points' slots); kMergeTail only positions >= k (the
// deferred tail).  Head and tail run with a.fuse_retire = 0: no slot writes here.
constexpr int kMergeAll = 0, kMergeHead = 1, kMergeTail = 2;
template <int BS, int KCAP, bool SC1, class Wait = MergeNoWait, int PART = kMergeAll>
__device__ __forceinline__ void merge_fused_block(const NestArgs& a, double* oll, long long* otie, int* oslot,
                                                  const int b, MergeLds<BS, KCAP>& L, const Wait& wait = Wait()) {
  [[maybe_unused]] constexpr int kMergeKid = PART == kMergeTail ? 2 : 3;   // trace stamps: tail apart
  const int64_t n = a.n, k = a.k, ns = n - k;
  const int nblk = (int)((ns + BS - 1) / BS);
  const int t = threadIdx.x;
  double* const s_sv_l = L.s_sv_l;
  long long* const s_sv_t = L.s_sv_t;
  double* const s_subl = L.s_subl;
  short* const s_sub = L.s_sub;
  short* const s_srt = L.s_srt;
  int* const s_scan = L.s_scan;
  constexpr int NW = BS / 64;                             // waves
  auto ldv = [](const auto* p) __attribute__((always_inline)) { return SC1 ? ld1(p) : *p; };
  const int64_t i0 = (int64_t)b * BS;
  const int nsb = (int)min((int64_t)BS, ns - i0);
  const double* sll = a.key_ll + k;
  const long long* stie = a.key_tie + k;
  const int* sslot = a.key_slot + k;
  const long long tie0 = -(long long)a.mrep - 1;          // tie of new key j: tie0 - j
  // loads: own survivor, the range's upper bound, the k new ll, and the first element of the
  // walkers' new points this thread copies into the slots they replace -- all in flight together
  // (the next walk reads the copied points after this kernel; nothing here reads them).  Element
  // g of the k x D block goes to thread g mod (nblk * BS) of the merge workgroups.
  const int64_t D = a.row_bytes / 8, kD = a.fuse_retire ? a.k * D : 0;
  const int64_t g0 = (int64_t)b * BS + t, gstride = (int64_t)nblk * BS;
  double kl = 0.0;
  long long kt = 0;
  int ks = 0;
  if (t < nsb) {
    kl = sll[i0 + t];
    kt = stie[i0 + t];
    ks = sslot[i0 + t];
  }
  const double lo_l = sll[i0];                            // the range: [s[i0], s[i0 + BS])
  const long long lo_t = stie[i0];
  const bool has_hi = i0 + BS < ns;
  const double hi_l = has_hi ? sll[i0 + BS] : 0.0;
  const long long hi_t = has_hi ? stie[i0 + BS] : 0;
  if (!wait()) return;
  int sj0 = 0;
  double cx0 = 0.0, cl0 = 0.0, cp0 = 0.0;
  int64_t d0 = -1;
  if (g0 < kD) {
    const int64_t j = g0 / D;
    d0 = g0 - j * D;
    sj0 = ldv(a.newk_slot + j);
    cx0 = ldv(a.nx + g0);
    if (d0 == 0) {
      cl0 = ldv(a.nll + j);
      cp0 = ldv(a.nlp + j);
    }
  }
  constexpr int kPer = KCAP / BS;
  double nv[kPer];
  int nsl[kPer];                                          // their slots: no global load after
#pragma unroll                                            // the subset is known
  for (int r = 0; r < kPer; ++r) {
    const int64_t j = (int64_t)r * BS + t;
    nv[r] = ldv(a.newk_ll + (j < k ? j : k - 1));
    nsl[r] = ldv(a.newk_slot + (j < k ? j : k - 1));
  }
  if (g0 < kD) {
    wt_store(&a.x[(int64_t)sj0 * D + d0], cx0);
    if (d0 == 0) {
      wt_store(&a.ll[sj0], cl0);
      wt_store(&a.lp[sj0], cp0);
    }
  }
  for (int64_t g = g0 + gstride; g < kD; g += gstride) {   // k * D beyond one element a thread
    const int64_t j = g / D;
    const int64_t d = g - j * D;
    const int sj = ldv(a.newk_slot + j);
    wt_store(&a.x[(int64_t)sj * D + d], ldv(a.nx + g));
    if (d == 0) {
      wt_store(&a.ll[sj], ldv(a.nll + j));
      wt_store(&a.lp[sj], ldv(a.nlp + j));
    }
  }
  // the new ll stay in registers: classified as they land, and only the block's subset goes to
  // LDS (no staging of all k of them, and no barrier before the classification)
  // classify this thread's new keys j = r * BS + t: below the range, or inside it.  Subset
  // offsets come from wave ballots (the r-th key of every lane: its rank among the wave's set
  // bits), the wave totals go through LDS; c_lo is summed the same way (integers: exact in any
  // order).  The subset order does not matter: it is ranked by counting below.
  uint32_t inmask = 0;
  int wsub = 0, wbelow = 0;                               // wave-uniform
#pragma unroll 16
  for (int r = 0; r < kPer; ++r) {
    const int64_t j = (int64_t)r * BS + t;
    const bool ok = j < k;
    const double x = nv[r];
    const long long xt = tie0 - j;
    const bool ge_lo = (b == 0) | !key_less(x, xt, lo_l, lo_t);
    const bool lt_hi = !has_hi | key_less(x, xt, hi_l, hi_t);
    const bool in = ok & ge_lo & lt_hi;
    inmask |= (in ? 1u : 0u) << r;
    wsub += __popcll(__ballot(in));
    wbelow += __popcll(__ballot(ok & !ge_lo));
  }
  NT_STAMP(kMergeKid, 1);
  if (t < nsb) {
    s_sv_l[t] = kl;
    s_sv_t[t] = kt;
  }
  const int lane = t & 63, wv = t >> 6;
  if (lane == 0) {
    s_scan[wv] = wsub;                                    // wave totals
    s_scan[NW + wv] = wbelow;
  }
  __syncthreads();
  int o = 0, m = 0;
  int64_t c_lo = 0;
#pragma unroll
  for (int w2 = 0; w2 < NW; ++w2) {
    o += w2 < wv ? s_scan[w2] : 0;
    m += s_scan[w2];
    c_lo += s_scan[NW + w2];
  }
#pragma unroll 16
  for (int r = 0; r < kPer; ++r) {
    const bool in = (inmask >> r) & 1u;
    const unsigned long long bm = __ballot(in);
    const int below_lane = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
    if (in) {
      s_sub[o + below_lane] = (short)(r * BS + t);
      s_subl[o + below_lane] = nv[r];
      L.s_subslot[o + below_lane] = nsl[r];
    }
    o += __popcll(bm);
  }
  __syncthreads();
  NT_STAMP(kMergeKid, 2);
  // rank the subset among itself (counting), place it sorted, write the subset keys out
  for (int e = t; e < m; e += BS) {
    const int j = s_sub[e];
    const double x = s_subl[e];
    const long long xt = tie0 - j;
    int lr = 0;
#pragma unroll 8
    for (int q = 0; q < m; ++q)                           // broadcast LDS reads, independent
      lr += key_less(s_subl[q], tie0 - s_sub[q], x, xt) ? 1 : 0;
    s_srt[lr] = (short)e;
    int lo = 0, hi = nsb;                                 // block survivors below x
    while (lo < hi) {
      const int md = (lo + hi) >> 1;
      if (key_less(s_sv_l[md], s_sv_t[md], x, xt)) lo = md + 1;
      else hi = md;
    }
    const int64_t pos = i0 + lo + c_lo + lr;
    if ((PART == kMergeTail && pos < k) || (PART == kMergeHead && pos >= k)) continue;
    wt_store(&oll[pos], x);
    wt_store(&otie[pos], xt);
    wt_store(&oslot[pos], L.s_subslot[e]);
    if (pos % kKeySample == kKeySample - 1) {
      a.out_samp_ll[pos / kKeySample] = x;
      a.out_samp_tie[pos / kKeySample] = xt;
    }
    if (PART == kMergeAll && pos == n - 1) {
      a.st->max_ll = x;
      __hip_atomic_fetch_add(&a.st->gen_done, 1LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  NT_STAMP(kMergeKid, 3);
  if (t < nsb) {                                          // survivors: i + c_lo + #subset below
    int lo = 0, hi = m;
    while (lo < hi) {
      const int md = (lo + hi) >> 1;
      const int em = s_srt[md];
      if (key_less(s_subl[em], tie0 - s_sub[em], kl, kt)) lo = md + 1;
      else hi = md;
    }
    const int64_t pos = i0 + t + c_lo + lo;
    if ((PART != kMergeTail || pos >= k) && (PART != kMergeHead || pos < k)) {
    wt_store(&oll[pos], kl);
    wt_store(&otie[pos], kt);
    wt_store(&oslot[pos], ks);
    if (pos % kKeySample == kKeySample - 1) {
      a.out_samp_ll[pos / kKeySample] = kl;
      a.out_samp_tie[pos / kKeySample] = kt;
    }
    }
    if (PART == kMergeAll && pos == n - 1) {
      a.st->max_ll = kl;
      __hip_atomic_fetch_add(&a.st->gen_done, 1LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  NT_STAMP(kMergeKid, 4);
}

// ---- split merge (round 6): the head of a generation's merge on the critical path, its tail
// deferred into the next walk's launch ----
//
// The next walk needs only the k lowest keys of the merged order (its threshold key[k-1], the
// slots key_slot[0..k) that its walkers retire and replace) and the stop test's inputs; walkers
// start at random live slots, not at sorted ranks.  Survivor block b of the merge writes
// positions >= B b, so blocks b < ceil(k / B) hold every position < k: the head kernel runs just
// those blocks (merge_fused_block<..., kMergeHead>), and the tail (kMergeTail, positions >= k,
// every block) runs in the workgroups of the next walk kernel behind its walkers.
constexpr int kHeadT = 512;                                // the head kernel's workgroup size
constexpr int kHeadR = kSmallSort / kHeadT;                // new keys per thread (L_max)

// the generation's L_max (the merged keys' last ll: the larger of the survivors' and the new keys'
// largest ll) and its count, after the estimate (same workgroup, k <= 4096)
__device__ __forceinline__ double head_lmax_load(const NestArgs& a) {   // issued before the estimate
  double mx = -__builtin_inf();
#pragma unroll
  for (int r = 0; r < kHeadR; ++r) {
    const int64_t j = r * kHeadT + threadIdx.x;
    if (j < a.k) mx = fmax(mx, a.newk_ll[j]);
  }
  return mx;
}
__device__ __forceinline__ void head_lmax(const NestArgs& a, double mx, double* s_red) {
  constexpr int T = kHeadT;
  const int t = threadIdx.x;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
  __syncthreads();
  if ((t & 63) == 0) s_red[t >> 6] = mx;
  __syncthreads();
  if (t == 0) {
    double M = a.st->max_ll;
#pragma unroll
    for (int w = 0; w < T / 64; ++w) M = fmax(M, s_red[w]);
    a.st->max_ll = M;
    a.st->gen_done = a.st->gen_done + 1;
  }
}
