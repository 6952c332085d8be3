// mcg_nested_kernel.h -- kernels of the batched nested sampler (Nested.nested_evidence,
// nested.ml:122-146) generalised to k retirements per generation.
//
// Device data:
//   live set     x[slot][D] (AoS rows: the DE proposal gathers two random rows per step),
//                ll[slot], lp[slot]
//   order        keys (ll, tie, slot) sorted ascending -- the k lowest are keys[0..k); the
//                reference's insertion-sorted array (nested.ml:26-43) becomes a merge of the
//                k sorted new keys into the n-k survivors each generation
//   dead points  dead_x[m][D], dead_ll[m], dead_lp[m] in retirement order
//   scalars      NestDevState (running log volume, estimate, stop / error flags)
#pragma once
#include "mcg_device.h"
#include "mcg_math.h"
#include "mcg_mh_kernel.h"
#include "mcg.h"

namespace mcg {

// log_vol / est are double-buffered by generation parity: generation g reads half g & 1 (its stop
// test, its dead points' log dv) and its estimate fold writes half (g + 1) & 1, so a fold that runs
// while generation g's walk is still reading (the split merge's in-walk estimate) never races it
struct NestDevState {
  double log_vol[2];
  double est[2];
  int32_t stopped;
  int32_t error;
  long long gen_done;
  double max_ll;            // the largest live ll (the sorted keys' last): the stop test's L_max
};

// The stop / error flags and the generation count are read and written with agent-scope atomics
// (sc1: past the L1 and scalar caches).  A kernel that read a stale stopped == 0 after the
// stopping generation would run a partial generation after the stop (seen with another process
// sharing the GPU: a retire kernel replaced live rows that the final keys no longer described).
__device__ __forceinline__ bool nest_stopped(const NestDevState* st) {
  return __hip_atomic_load(&st->stopped, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
__device__ __forceinline__ void nest_set(int32_t* flag) {
  __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// last-workgroup hand-off counters (mcg_nested_kernels.hip, last_block_done): per use a top counter
// and 16 group counters, each on a 128-B line of its own; every counter is reset by the workgroup
// that completes it
constexpr int kKeySample = 64;   // spacing of the sorted-key sample kept beside the keys
constexpr int kSyncGroups = 16, kSyncStride = 32, kSyncUse = (kSyncGroups + 1) * kSyncStride;

struct NestArgs {
  MhArgs m;                 // likelihood / prior constants (m.lik, m.pri, m.prior_kind, ...)
  double* x;                // live rows [n][D]
  double* ll;
  double* lp;
  const double* key_ll;     // current sorted keys
  const long long* key_tie;
  const int* key_slot;
  const double* key_samp_ll;    // every kKeySample-th current key (written by the previous merge)
  const long long* key_samp_tie;
  double* out_samp_ll;          // the same sample of the merged keys, for the next generation
  long long* out_samp_tie;
  double* nx;               // new points [k][D]
  double* nll;
  double* nlp;
  double* dead_x;
  double* dead_ll;
  double* dead_lp;
  // the batch's host staging (pinned, coherent, device-mapped): each retirement's ll / lp also go
  // straight to host memory at index m - h_m0, so a batch needs no copy of them (null: none)
  double* h_ll;
  double* h_lp;
  int64_t h_m0;
  double* newk_ll;          // unsorted keys of the new points
  long long* newk_tie;
  int* newk_slot;
  int* rank;                // [k] rank of new key j among the generation's new keys (k <= 4096)
  uint32_t* sync;           // [2][kSyncUse] hand-off counters: retire -> estimate, rank count -> scatter
  unsigned long long* trace;  // MCG_NEST_TRACE builds: per-workgroup phase stamps of one generation
  // the walkers' draws of a generation, [2][nmcmc][k] (null: the walk draws them itself): DE
  // pair as row byte offsets (i | j << 32) * row_bytes and (DE scale, log accept uniform).  The walk of generation g reads half
  // g & 1 while its spare waves fill the other half for generation g + 1.
  unsigned long long* rt_ix;
  double2* rt_sc;
  int32_t est_in_rank;      // the estimate is folded by an extra rank_count workgroup (k <= 4096)
  int32_t fuse_retire;      // (k <= 4096) no retire kernel: each walker retires its own dead point
                            // at its start and emits its key at its end; the rank-count workgroups
                            // put the new points into the freed slots
  int32_t sym_box;          // box prior with lo[d] == -hi[d] for every d: tested as |y| <= hi
  int32_t lanes_hint;       // lanes per walker requested by MCG_NEST_LANES (0: the default)
  int32_t walk_waves;       // walker waves per draw-table workgroup (1, or 2 beyond 256 waves)
  // the merge role of the walk kernel (k <= 4096 with the draw table): workgroups past the
  // walkers' nwalk_blocks wait for their go flag, then merge the new keys into mrg_*
  // (merge_fused_block) or fold the estimate
  int32_t fuse_merge;
  int32_t nwalk_blocks;
  uint32_t* fm_sync;        // [16 group counters | top counter | go flag per merge workgroup], 128 B apart
  double* mrg_ll;
  long long* mrg_tie;
  int* mrg_slot;
  // split merge (round 6): the head kernel writes the merged keys [0, k); the
  // tail (positions >= k) of generation g runs in walk g + 1's launch, in tl_nblk workgroups past
  // its nwalk_blocks walker workgroups (0: none), from generation g's inputs below, and only when
  // generation g's head ran (gen_done >= tl_gen1)
  int32_t split;
  int32_t est_in_walk;      // split merge: the generation's estimate is folded during its walk by
                            // one workgroup past the tail's, once every table-filling wave has
                            // stored its dead points' tv (counter a.sync[0])
  int32_t tl_nblk;
  int64_t tl_mrep, tl_gen1;
  const double* tl_key_ll;  // generation g's keys (the merge's input)
  const long long* tl_key_tie;
  const int* tl_key_slot;
  double* tl_newk_ll;       // generation g's new keys (double-buffered by generation parity)
  int* tl_newk_slot;
  double* tl_out_ll;        // the merged keys (this walk's keys: positions >= k)
  long long* tl_out_tie;
  int* tl_out_slot;
  double* tl_samp_ll;
  long long* tl_samp_tie;
  uint32_t row_bytes;       // D * 8: the draw table holds DE pairs as row byte offsets
  double* tv;               // ll + log dv of this generation's dead points (padded pow2)
  const double* prefix;     // [k+1] sum_{j'<j} log1p(-1/(n-j'))
  const double* qadd;       // [k] 1/(n-j) (nested.ml:140 quirk) or log(1/(n-j))
  NestDevState* st;
  int64_t n, k, nmcmc, mrep, tv_len;
  double mode_hop, sigma_de, log_epsrel;
  uint32_t k0, k1;
  uint64_t seed_unused;
};

// phase stamps (s_memrealtime, 100 MHz) of wave 0 of each workgroup, one generation, in
// MCG_NEST_TRACE builds only: trace[(kernel * 1024 + block) * 8 + slot]
#ifdef MCG_NEST_TRACE
#define NT_STAMP(kid, slot)                                                                       \
  do {                                                                                            \
    if (a.trace && threadIdx.x == 0 && blockIdx.x < 1024)                                         \
      a.trace[((size_t)(kid) * 1024 + blockIdx.x) * 8 + (slot)] = wall_clock64();                 \
  } while (0)
#else
#define NT_STAMP(kid, slot) do {} while (0)
#endif

__device__ __forceinline__ int gen_par(const NestArgs& a) { return (int)((a.mrep / a.k) & 1); }

// one retirement's ll / lp into the dead buffers and, when the batch stages on the host, into the
// pinned staging buffers (posted writes over PCIe; the host reads them after the batch's event)
__device__ __forceinline__ void put_dead(const NestArgs& a, int64_t m, double ll, double lp) {
  a.dead_ll[m] = ll;
  a.dead_lp[m] = lp;
  if (a.h_ll) {
    a.h_ll[m - a.h_m0] = ll;
    a.h_lp[m - a.h_m0] = lp;
  }
}

// an output store read by a later kernel as sc1 (a relaxed agent-scope atomic store: written
// through and dropped from the XCD's L2, so less is left to write back when the kernel ends);
// the fused merge's outputs
template <class T>
__device__ __forceinline__ void wt_store(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kNestPrefetch = 4;                   // DE steps whose partner rows are in flight
// pad rows per draw-table half: the walker loads entries up to 3 prefetch groups past its step
constexpr int kWalkTabPad = 3 * kNestPrefetch;
constexpr int kNestWalkBlock = 64;

// The random numbers of walker step s (draw_new_live_point, nested.ml:50-74): the DE pair i != j
// (pick_samples, mcmc.ml:199-203), the DE scale (1 with probability mode_hop, else
// N(0, 2.38/sqrt(2D)), mcmc.ml:209-213) and log u of the accept test (mcmc.ml:49).  LU = false:
// the walker's accept test never reads log u (the shell walker, see its step), left 0
template <bool LU = true>
__device__ __forceinline__ void walk_draw(const NestArgs& a, uint32_t wid, uint32_t s,
                                          const double2* nt, const double2* lt,
                                          unsigned long long& ix, double2& sc) {
  const Rng rng{a.k0, a.k1};
  const uint32_t n = (uint32_t)a.n;
  const u32x4 rI = rng(wid, s, CALL_DE_IDX, TAG_NEST_WALK, 0u);
  const u32x4 rS = rng(wid, s, CALL_DE_SCALE, TAG_NEST_WALK, 0u);
  const uint32_t i = randint(rI.x, rI.y, n);
  const uint32_t jj = randint(rI.z, rI.w, n - 1);
  const uint32_t j = jj + (jj >= i ? 1u : 0u);
  ix = (unsigned long long)i | ((unsigned long long)j << 32);
  sc.x = (a.mode_hop != 0.0 && u53(rS.x, rS.y) < a.mode_hop) ? 1.0 : a.sigma_de * pnormal(rS.z, nt);
  if constexpr (LU) {
    const u32x4 rA = rng(wid, s, CALL_ACCEPT, TAG_NEST_WALK, 0u);
    sc.y = plog(u53(rA.x, rA.y), lt);
  } else {
    sc.y = 0.0;
  }
}

// the draws of every walker step of the generation that starts at replacement mrep, entries
// [e0, k nmcmc) with stride `stride` (layout [step][walker])
// Generation g = mrep / k uses half g & 1 of the double-buffered table.  Each half has
// nmcmc + kWalkTabPad rows of k entries: the pad rows (zero: DE pair (0, 0), scale 0, log u 0,
// written once at allocation) serve the walker's look-ahead loads past the last step, which
// therefore need no clamp.
__device__ __forceinline__ int64_t walk_tab_base(const NestArgs& a, int64_t mrep) {
  return ((mrep / a.k) & 1) * a.k * (a.nmcmc + kWalkTabPad);
}
template <bool LU = true>
__device__ __forceinline__ void walk_draws_fill(const NestArgs& a, int64_t mrep, int64_t e0, int64_t stride,
                                                const double2* lt) {
  const int64_t tot = a.k * a.nmcmc, base = walk_tab_base(a, mrep);
  for (int64_t e = e0; e < tot; e += stride) {
    const int64_t s = e / a.k, w = e - s * a.k;
    unsigned long long ix;
    double2 sc;
    walk_draw<LU>(a, (uint32_t)(mrep + w), (uint32_t)s, kNrmTab, lt, ix, sc);
    // byte offsets of the two rows: the walker adds them to the live set's base with no 64-bit
    // address arithmetic
    ix = (unsigned long long)((uint32_t)ix * a.row_bytes) | ((unsigned long long)((uint32_t)(ix >> 32) * a.row_bytes) << 32);
    a.rt_ix[base + e] = ix;
    a.rt_sc[base + e] = sc;
  }
}

// Lane layout of a walker on P lanes: lane `sub` owns the W-dim blocks c = sub, sub + P, ...
// (dims W c .. W c + W - 1).  W = 4 is the MH kernel's Layout (Philox blocks); W = 2 when D = 2P
// (D = 8 on 4 lanes, D = 16 on 8), whose lanes each hold two dims: the two lanes of a canonical
// accumulator (dims 4j .. 4j + 3, DESIGN.md §Canonical sums) then chain their fmas in dim order
// (reduce_canon_w2).  The walker's DE proposal draws no per-dim random numbers, so any split of
// the dims is the same computation.
template <int D, int P>
struct WalkLayout {
  static constexpr int W = (P > 1 && D == 2 * P) ? 2 : 4;
  static constexpr int NC = (D + W - 1) / W;               // blocks
  static constexpr int NCL = (NC + P - 1) / P;             // blocks owned by one lane
  static constexpr int NL = NCL * W;                       // local dims
  static constexpr int NA = W == 2 ? 1 : 8 / P;            // local accumulators (W = 4)
  static_assert(P == 1 || P == 2 || P == 4 || P == 8, "P must divide 8");
  static_assert(P == 1 || D % (W * P) == 0, "P > 1 needs D % WP == 0");
  __device__ static __forceinline__ int dim(int sub, int i, int q) { return W * (sub + P * i) + q; }
  __device__ static __forceinline__ bool valid(int sub, int i, int q) {
    return q < W && (P > 1 || (W * i + q) < D);
  }
};

// (the canonical sum for W = 2 is reduce_canon_w2, mcg_mh_kernel.h)

// The log-target constants of one walker lane (its dims of mu/sigma or the shell centre, the box
// bounds), loaded into registers once per launch.  Loaded per step through the parameter
// pointers they would queue behind the prefetched DE rows in the in-order vector-memory counter
// and expose the full load latency every step.  Same operations as eval_lik / eval_prior.
template <int D, int P, int LIK, bool SYM = false, bool GP = false>
struct WalkTarget {
  using Lay = WalkLayout<D, P>;
  static constexpr int W = Lay::W;
  static constexpr int NL = Lay::NL;
  static constexpr bool kReg =
      (LIK == MCG_LIK_DIAG_GAUSS || LIK == MCG_LIK_GAUSS_SHELL || LIK == MCG_LIK_FLAT) && NL <= 8;
  static constexpr int NR = kReg ? NL : 1;
  double m0[NR], m1[NR], lo[NR], hi[NR];
  double c0 = 0.0, c1 = 0.0, c2 = 0.0, lp_in = 0.0;
  bool box = false;

  __device__ __forceinline__ void load(const MhArgs& a, int sub) {
    if constexpr (kReg) {
      const double* __restrict__ q = a.lik;
      const double* __restrict__ pr = a.pri;
      box = !GP && a.prior_kind != MCG_PRIOR_FLAT;   // GP: no bounds (lo, hi = -+inf)
#pragma unroll
      for (int i = 0; i < Lay::NCL; ++i)
#pragma unroll
        for (int k = 0; k < W; ++k) {
          const int j = W * i + k;
          const bool v = Lay::valid(sub, i, k);
          const int d = v ? Lay::dim(sub, i, k) : 0;
          m0[j] = (v && LIK != MCG_LIK_FLAT) ? q[d] : 0.0;
          m1[j] = (v && LIK == MCG_LIK_DIAG_GAUSS) ? q[D + d] : 0.0;
          lo[j] = (v && !GP) ? pr[d] : -__builtin_inf();
          hi[j] = (v && !GP) ? pr[D + d] : __builtin_inf();
        }
      if constexpr (LIK == MCG_LIK_DIAG_GAUSS) c0 = q[2 * D];
      if constexpr (LIK == MCG_LIK_GAUSS_SHELL) { c0 = q[D]; c1 = q[D + 1]; c2 = q[D + 2]; }
      lp_in = GP ? 0.0 : pr[2 * D];
    }
  }

  __device__ __forceinline__ double lik(const double* y, int sub, const MhArgs& a) const {
    if constexpr (!kReg) {
      return eval_lik<D, P, LIK>(y, sub, a, a.lik);
    } else if constexpr (LIK == MCG_LIK_FLAT) {
      return 0.0;
    } else {
      double S;
      if constexpr (W == 2) {
        double e[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          e[j] = LIK == MCG_LIK_DIAG_GAUSS ? fma(y[j], m1[j], -m0[j]) : y[j] - m0[j];
        S = reduce_canon_w2<P>(e[0], e[1], sub);
      } else {
        double A[Lay::NA];
#pragma unroll
        for (int j = 0; j < Lay::NA; ++j) A[j] = 0.0;
#pragma unroll
        for (int i = 0; i < Lay::NCL; ++i)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (!Lay::valid(sub, i, k)) continue;
            const int j = 4 * i + k;
            double e;
            if constexpr (LIK == MCG_LIK_DIAG_GAUSS) e = fma(y[j], m1[j], -m0[j]);
            else e = y[j] - m0[j];
            A[i % Lay::NA] = fma(e, e, A[i % Lay::NA]);
          }
        S = reduce_canon<P>(A);
      }
      if constexpr (LIK == MCG_LIK_DIAG_GAUSS) {
        return c0 - 0.5 * S;
      } else {
        const double r = psqrt(S);
        const double qq = (r - c0) * c1;
        return c2 - 0.5 * qq * qq;
      }
    }
  }

  // SHELL: the step's constraint test lik(y) >= thr decided on S = |y - c|^2, off the sqrt:
  // S in [s_in_lo, s_in_hi] passes, S below s_out_lo or above s_out_hi fails, and only S in the
  // guard bands between is evaluated exactly (lik, psqrt).  The bands are ~1e-9 r wide plus a
  // bound on the exact evaluation's rounding, so both routes give the same answer.
  double s_in_lo = 0.0, s_in_hi = 0.0, s_out_lo = 0.0, s_out_hi = 0.0;

  __device__ __forceinline__ void setup_constraint(double thr) {
    if constexpr (kReg && LIK == MCG_LIK_GAUSS_SHELL) {
      const double inf = __builtin_inf();
      const double g = c2 - thr;                     // lik <= c2 everywhere
      if (!(g >= 0.0) || !(c1 > 0.0) || !(c0 >= 0.0)) {
        s_in_lo = inf; s_in_hi = -inf;               // nothing definitely passes
        s_out_lo = g >= 0.0 ? -inf : inf;            // g < 0: everything fails, else exact
        s_out_hi = g >= 0.0 ? inf : -inf;
        return;
      }
      const double delta = sqrt(2.0 * g) / c1;       // lik = thr at r = c0 -+ delta
      const double df = 64.0 * 2.220446049250313e-16 * (fabs(c2) + fabs(thr) + 1.0);
      const double dr = fmax(df / (c1 * c1 * fmax(delta, 1e-300)), sqrt(2.0 * df) / c1);
      const double band = 1e-9 * (c0 + delta) + 4.0 * dr;
      const double r_lo = c0 - delta, r_hi = c0 + delta;
      const double a_lo = fmax(r_lo + band, 0.0), a_hi = r_hi - band;
      if (a_hi >= a_lo) { s_in_lo = a_lo * a_lo; s_in_hi = a_hi * a_hi; }
      else { s_in_lo = inf; s_in_hi = -inf; }
      s_out_lo = (r_lo - band > 0.0) ? (r_lo - band) * (r_lo - band) : -inf;
      s_out_hi = (r_hi + band) * (r_hi + band);
      // A point the band test can pass has S <= s_out_hi, so each |y_k - c_k| <= sqrt(S) up to
      // the sum's rounding (< 1e-14 relative at D <= 64).  Once the box holds that whole ball
      // (late generations: the shell well inside the prior box), no such point is outside the
      // box and the box test cannot change a decision: the walk skips it (wave-uniform).
      {
        const double R = sqrt(s_out_hi) * (1.0 + 1e-9) + 1e-300;
        bool ok = s_out_hi >= 0.0 && R < inf;
#pragma unroll
        for (int j = 0; j < NL; ++j) {
          if constexpr (SYM) ok = ok && (__builtin_fabs(m0[j]) + R <= hi[j]);
          else ok = ok && (m0[j] - R >= lo[j]) && (m0[j] + R <= hi[j]);
        }
        box_test = __ballot(!ok) != 0;
      }
    }
  }
  bool box_test = true;

  // lik(y) >= thr, exactly as the comparison of the evaluated likelihood (mcmc_logl, nested.ml:54-59)
  __device__ __forceinline__ bool constraint(const double* y, int sub, const MhArgs& a, double thr) const {
    if constexpr (kReg && LIK == MCG_LIK_GAUSS_SHELL) {
      double S;
      if constexpr (W == 2) {
        S = reduce_canon_w2<P>(y[0] - m0[0], y[1] - m0[1], sub);
      } else {
        double A[Lay::NA];
#pragma unroll
        for (int j = 0; j < Lay::NA; ++j) A[j] = 0.0;
#pragma unroll
        for (int i = 0; i < Lay::NCL; ++i)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (!Lay::valid(sub, i, k)) continue;
            const int j = 4 * i + k;
            const double e = y[j] - m0[j];
            A[i % Lay::NA] = fma(e, e, A[i % Lay::NA]);
          }
        S = reduce_canon<P>(A);
      }
      bool in = (S >= s_in_lo) & (S <= s_in_hi);
      const bool out = (S < s_out_lo) | (S > s_out_hi);
      if (!(in | out)) {                             // guard band (rare): the exact evaluation
        const double r = psqrt(S);
        const double qq = (r - c0) * c1;
        in = (c2 - 0.5 * qq * qq) >= thr;
      }
      return in;
    } else {
      return lik(y, sub, a) >= thr;
    }
  }

  // The step's constraint and box prior as ONE cross-lane reduction: a lane
  // outside the box adds NaN to one of its canonical accumulators, inside it adds 0.0.  Every
  // accumulator is a sum of squares started from +0.0, so x + 0.0 = x and S keeps its bits; a
  // NaN makes S NaN, which the band test below counts as outside (!(S >= lo) is true for NaN),
  // so the step rejects for any threshold -- as prior() = -inf would.  Inside the box the
  // decision is constraint() && prior() > -inf exactly.  W = 4 register targets (the shell).
  static constexpr bool kFold = kReg && LIK == MCG_LIK_GAUSS_SHELL && W == 4 && !GP;
  __device__ __forceinline__ double lp_box() const { return (SYM || box) ? lp_in : 0.0; }
  template <bool BOXT = true>   // BOXT = false: the box test is implied (box_test false)
  __device__ __forceinline__ bool constraint_box(const double* y, int sub, double thr) const {
    double A[Lay::NA];
#pragma unroll
    for (int j = 0; j < Lay::NA; ++j) A[j] = 0.0;
#pragma unroll
    for (int i = 0; i < Lay::NCL; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!Lay::valid(sub, i, k)) continue;
        const int j = 4 * i + k;
        const double e = y[j] - m0[j];
        A[i % Lay::NA] = fma(e, e, A[i % Lay::NA]);
      }
    if (BOXT && (SYM || box)) {
      int inb = 1;
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        if constexpr (SYM) inb &= (int)(__builtin_fabs(y[j]) <= hi[j]);
        else inb &= (int)(y[j] >= lo[j]) & (int)(y[j] <= hi[j]);
      }
      const double pen = inb ? 0.0 : __builtin_nan("");
      A[Lay::NA - 1] = A[Lay::NA - 1] + pen;
    }
    const double S = reduce_canon<P>(A);
    bool in = (S >= s_in_lo) & (S <= s_in_hi);
    const bool out = !(S >= s_out_lo) | !(S <= s_out_hi);   // NaN: out
    if (!(in | out)) {                               // guard band (rare): the exact evaluation
      const double r = psqrt(S);
      const double qq = (r - c0) * c1;
      in = (c2 - 0.5 * qq * qq) >= thr;
    }
    return in;
  }

  __device__ __forceinline__ double prior(const double* y, int sub, const MhArgs& a) const {
    if constexpr (GP) {
      // Stats.log_multi_gaussian of the prior (canonical DIAG form), its constants through
      // scalar loads (kept out of the in-order vector-memory queue of the prefetched DE rows)
      typedef const __attribute__((address_space(4))) double kconst;
      kconst* kpri = (kconst*)a.pri;
      asm volatile("" : "+s"(kpri));
      return eval_gauss_prior<D, P, kconst*, W>(y, sub, a, kpri);
    } else if constexpr (!kReg) {
      return eval_prior<D, P>(y, sub, a, a.pri);
    } else {
      if (!SYM && !box) return 0.0;                   // SYM implies a box prior
      int inb = 1;
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        // SYM: |y| <= h is the same predicate as -h <= y <= h for every double, NaN included
        if constexpr (SYM) inb &= (int)(__builtin_fabs(y[j]) <= hi[j]);
        else inb &= (int)(y[j] >= lo[j]) & (int)(y[j] <= hi[j]);
      }
      inb = and_lanes<P>(inb);
      return inb ? lp_in : -__builtin_inf();
    }
  }
};

#include "mcg_nested_merge.h"

// ---- constrained DE-MCMC walkers (draw_new_live_point, nested.ml:50-74) ----
// P lanes per walker (P in {1, 2, 4}; the MH kernel's layout: lane `sub` owns the 4-dim blocks
// c = sub, sub + P, ...).  Every lane of a walker draws the same Philox words, so the DE indices,
// scale, accept decision and start point agree without communication; the log-target is the
// canonical sum reduced across the P lanes (reduce_canon).  The DE partner rows of step s + 1
// depend only on the RNG, so they are loaded while step s computes (one step of prefetch).
// The merge role of a fused walk kernel (FM): workgroup b = blockIdx.x - nwalk_blocks of the
// generation's merge (b == nblk: the estimate fold).  Hand-off (row 1 of MI355X_MICROARCH.md's
// hand-offs): every walker workgroup stores its outputs sc1, waits vmcnt(0), passes a barrier and
// adds to its group counter (16 counters on 128-B lines of their own, then a top counter); the
// workgroup that completes the top counter writes each merge workgroup's go flag (own 128-B line,
// the generation number).  A merge workgroup polls only its flag -- or the stop / error flags: a
// generation the walkers stop never signals -- then runs merge_fused_block with sc1 loads of the
// walkers' outputs.  It reads none of the stop test's inputs (log_vol, est, max_ll), which the
// estimate and the last key's workgroup rewrite in this launch.  The wait is bounded: past ~1 s
// it flags an error (the host then reports a failed run) instead of hanging the grid.
__device__ __forceinline__ uint32_t* fm_go(const NestArgs& a, int b) {
  return a.fm_sync + (size_t)(kSyncGroups + 1 + b) * kSyncStride;
}

__device__ __forceinline__ void nest_merge_role(const NestArgs& a) {
  constexpr int BS = 256, KCAP = kSmallSort;
  const int b = (int)blockIdx.x - a.nwalk_blocks;
  const int nblk = (int)((a.n - a.k + BS - 1) / BS);
  if (b > nblk) return;
  NT_STAMP(3, 0);
  if (nest_stopped(a.st)) return;                       // stopped in an earlier launch
  __shared__ union FmLds {
    MergeLds<BS, KCAP> m;
    EstLds<BS> e;
  } lds;
  __shared__ int s_ok;
  // the hand-off: one thread polls the go flag, the workgroup waits at a barrier
  auto wait = [&]() -> bool {
    if (threadIdx.x == 0) {
      const uint32_t gen1 = (uint32_t)(a.mrep / a.k + 1);
      const uint32_t* go = fm_go(a, b);
      int ok = 0;
      for (uint32_t it = 0;; ++it) {
        if (ld1(go) >= gen1) {
          ok = 1;
          break;
        }
        if (nest_stopped(a.st) || __hip_atomic_load(&a.st->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
        if (it > (1u << 22)) {
          // the hand-off's own error code (2): reported as a timeout, not as a failed draw
          __hip_atomic_store(&a.st->error, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      s_ok = ok;
    }
    __syncthreads();
    NT_STAMP(3, 5);
    return s_ok != 0;
  };
  if (b == nblk) {
    if (wait()) estimate_body<BS>(a, lds.e);
  } else {
    // the survivors' keys (the previous launch's output) are loaded before the wait
    merge_fused_block<BS, KCAP, true>(a, a.mrg_ll, a.mrg_tie, a.mrg_slot, b, lds.m, wait);
  }
}

// The deferred tail of generation g's merge (split merge): survivor block b of the BS = 256
// partition (the walk kernel's workgroup size), positions >= k only.  It reads nothing this
// launch's walkers write (generation g's keys and new keys; the walkers write generation g + 1's
// new keys into the other half) and writes positions the walkers do not read (they read [0, k)).
__device__ __forceinline__ void nest_tail_block(const NestArgs& a, int b) {
  if (__hip_atomic_load(&a.st->gen_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.tl_gen1) return;
  NestArgs t = a;
  t.key_ll = a.tl_key_ll;
  t.key_tie = a.tl_key_tie;
  t.key_slot = a.tl_key_slot;
  t.newk_ll = a.tl_newk_ll;
  t.newk_slot = a.tl_newk_slot;
  t.mrep = a.tl_mrep;
  t.out_samp_ll = a.tl_samp_ll;
  t.out_samp_tie = a.tl_samp_tie;
  t.fuse_retire = 0;
  __shared__ MergeLds<256, kSmallSort> ml;
  merge_fused_block<256, kSmallSort, false, MergeNoWait, kMergeTail>(t, a.tl_out_ll, a.tl_out_tie, a.tl_out_slot, b, ml);
}

// The split merge's estimate of generation g, folded inside walk g: the workgroup past the tail's
// makes the generation's stop test (as every walk workgroup does; a stopping generation retires
// nothing), waits until every table-filling wave has stored its tv (a.sync[0] counts them; bounded,
// error 2 past ~1 s) and folds est / log_vol into half (g + 1) & 1 -- which this generation's
// stop test and tv never read.  Off the generation's serial path: the walk runs ~20 us, the tv
// stores land in the first ~2.
__device__ __forceinline__ void nest_est_role(const NestArgs& a, uint32_t nfill) {
  if (nest_stopped(a.st)) return;
  if (a.mrep > 0) {
    const int g = gen_par(a);
    const double live = a.st->log_vol[g] + a.st->max_ll;
    const bool err = __hip_atomic_load(&a.st->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (live - plse(a.st->est[g], live, kLogTab) <= a.log_epsrel || err) return;
  }
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    int ok = 0;
    for (uint32_t it = 0;; ++it) {
      if (ld1(a.sync) >= nfill) {
        ok = 1;
        break;
      }
      if (__hip_atomic_load(&a.st->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
      if (it > (1u << 22)) {
        __hip_atomic_store(&a.st->error, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    if (ok) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    s_ok = ok;
  }
  __syncthreads();
  if (!s_ok) return;
  __shared__ EstLds<256> el;
  estimate_body<256>(a, el);
  if (threadIdx.x == 0) st1(a.sync, 0u);                 // (the only reader: reset for walk g + 1)
}

// a walker workgroup of a fused walk kernel (FM) signals once every one of its waves has
// finished its stores (stored sc1 where the merge reads them); the last one sets the go flags
__device__ __forceinline__ void nest_walk_signal(const NestArgs& a) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const uint32_t gen1 = (uint32_t)(a.mrep / a.k + 1);
  if (threadIdx.x == 0) {
    const int nwb = a.nwalk_blocks, g = (int)blockIdx.x % kSyncGroups;
    const uint32_t members = (uint32_t)((nwb - g + kSyncGroups - 1) / kSyncGroups);
    const uint32_t ng = (uint32_t)min(nwb, kSyncGroups);
    int last = 0;
    if (__hip_atomic_fetch_add(a.fm_sync + (size_t)g * kSyncStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 ==
        gen1 * members)
      last = __hip_atomic_fetch_add(a.fm_sync + (size_t)kSyncGroups * kSyncStride, 1u, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT) + 1 == gen1 * ng;
    s_last = last;
  }
  __syncthreads();
  if (s_last) {
    const int nblk = (int)((a.n - a.k + 255) / 256);
    for (int b = threadIdx.x; b <= nblk; b += blockDim.x) st1(fm_go(a, b), gen1);
  }
}

// GP: a DIAG_GAUSS prior, whose log density makes the walker's MH test log u < lp(y) - lp(cur)
// (nested.ml:54-59) a real test (with box priors it holds for every passing proposal).
// FM: the generation's merge runs in the same launch (nest_merge_role), by the workgroups past
// the walkers' (TAB only, k <= 4096: one walker wave per workgroup)
template <int D, int LIK, int P, bool TAB, bool SYM, bool GP = false, bool FM = false>
__global__ void __launch_bounds__(256) nest_walk_kernel(const NestArgs a) {
  static_assert(!FM || TAB, "the fused merge needs the draw table's workgroup shape");
  if constexpr (FM) {
    if ((int)blockIdx.x >= a.nwalk_blocks) {
      nest_merge_role(a);
      return;
    }
  } else if constexpr (TAB) {
    if ((int)blockIdx.x >= a.nwalk_blocks) {            // split merge: the estimate, the previous tail
      // (the estimate's workgroup right behind the walkers': dispatched in order, it is placed
      // before the tail's ~500 workgroups queue for CUs)
      const int b = (int)blockIdx.x - a.nwalk_blocks - a.est_in_walk;
      if (b < 0) nest_est_role(a, (uint32_t)(a.nwalk_blocks * (4 - a.walk_waves)));
      else nest_tail_block(a, b);
      return;
    }
  }
  using Lay = WalkLayout<D, P>;
  constexpr int NL = Lay::NL;
  constexpr int W = Lay::W;
  NT_STAMP(0, 0);
  __shared__ double2 s_lt[kLogTabN];                 // math tables staged in LDS (gathers)
  const double2* nt = kNrmTab;   // (an LDS copy costs more to stage than its gathers save: 62 vs 52 us)
  // The walker wave's first loads go out before the table staging and the stop test, so their
  // latencies overlap instead of queueing one behind the other: the stop-test state, the
  // target constants, the threshold, the retired slot, the first start candidate's ll / lp / row (accepted ~(n - k) / n
  // of the time; the search below only runs when it fails), and with the draw table the first
  // group's draws and the partner-row indices of the ring.  All are plain reads of buffers the
  // previous kernels finished.
  const bool stopped0 = nest_stopped(a.st);
  const double st_lv = a.st->log_vol[gen_par(a)], st_mx = a.st->max_ll, st_est = a.st->est[gen_par(a)];
  const bool st_err = __hip_atomic_load(&a.st->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  // with the draw table a 256-thread workgroup holds ww walker waves (waves 0 .. ww-1, one SIMD
  // each) and 4 - ww table-filling waves: one walker wave per SIMD of the chip up to 1,024
  // walker waves (k P <= 65,536 lanes; ww = 2 from 256 walker waves on)
  const int ww = TAB ? a.walk_waves : 1;
  const int wl = 64 * ww;                              // walker lanes per workgroup
  const bool walker = !TAB || (int)threadIdx.x < wl;   // wave-uniform
  const int64_t tid = (int64_t)blockIdx.x * (TAB ? wl : blockDim.x) + threadIdx.x;
  const int sub = (int)(tid & (P - 1));
  const int64_t w = tid / P;
  const bool active = w < a.k;
  // inactive lanes of a partial wave run walker 0's arithmetic (shuffle partners) but store nothing
  const int64_t wc = active ? w : 0;
  const Rng rng{a.k0, a.k1};
  const uint32_t wid = (uint32_t)(a.mrep + wc);
  const uint32_t n = (uint32_t)a.n;
  constexpr int PD = kNestPrefetch;
  const int64_t tbase = TAB ? walk_tab_base(a, a.mrep) : 0;
  // per-lane entry pointers; step st (clamped to the last step) is at [st * k].  32-bit offsets
  // (the table is skipped beyond 512 MB, so k nmcmc < 2^25): as 64-bit products with the clamp
  // compare in VALU the eight entry addresses of a group cost ~80 SALU/VALU per group, issued by
  // the walker's single wave on its SIMD
  const double2* const tsc_lane = a.rt_sc + tbase + wc;
  const unsigned long long* const tix_lane = a.rt_ix + tbase + wc;
  const uint32_t tk = (uint32_t)a.k;
  auto tab_off = [&](int64_t st) -> uint32_t { return (uint32_t)st * tk; };   // pad rows: no clamp
  double thr = 0.0, ll_first = -__builtin_inf(), lp_first = 0.0;
  int ret_slot = 0;
  uint32_t s_first = 0;
  double row_first[NL];
  unsigned long long tix_cur[PD], tix_ring[PD];
  double2 tsc_cur[PD];
  using Tgt = WalkTarget<D, P, LIK, SYM, GP>;
  Tgt tgt;                                           // the log-target's constants (registers)
  if (walker) {
    tgt.load(a.m, sub);
    thr = a.key_ll[a.k - 1];
    ret_slot = a.key_slot[wc];                         // the live slot walker w's point replaces
    const u32x4 r = rng(wid, 0u, CALL_START, TAG_NEST_WALK, 0u);
    s_first = randint(r.x, r.y, n);
    ll_first = a.ll[s_first];
    lp_first = a.lp[s_first];
    const double* __restrict__ src = a.x + (int64_t)s_first * D;
#pragma unroll
    for (int i = 0; i < Lay::NCL; ++i)
#pragma unroll
      for (int q = 0; q < W; ++q)
        row_first[W * i + q] = Lay::valid(sub, i, q) ? src[Lay::dim(sub, i, q)] : 0.0;
    if constexpr (TAB) {
#pragma unroll
      for (int u = 0; u < PD; ++u) {
        tix_ring[u] = tix_lane[tab_off(u)];
        tsc_cur[u] = tsc_lane[tab_off(u)];
        tix_cur[u] = tix_lane[tab_off(PD + u)];
      }
    }
  }
  // the log table: staged in LDS for the walkers that draw their own numbers; with the draw
  // table the walkers need it only for the stop test and the filling waves gather from the
  // global copy (as they do for the normal table), so there is no staging barrier to wait for
  const double2* const lt = TAB ? kLogTab : s_lt;
  if constexpr (!TAB) {
    for (int i = threadIdx.x; i < kLogTabN; i += blockDim.x) s_lt[i] = kLogTab[i];
    __syncthreads();
  }
  NT_STAMP(0, 1);
  if (stopped0) return;
  if (a.mrep > 0) {
    // the previous generation's stop test (remaining_integral_negligable, nested.ml:45-48, on the
    // max live ll; or a failed draw, nested.ml:70-72), made by every workgroup from the same
    // inputs: a flag set inside a kernel could be seen by only some of its workgroups (a late
    // starter would skip its share of the work), so no kernel reads the flag it may set
    const double live = st_lv + st_mx;
    const bool err = st_err;
    if (live - plse(st_est, live, lt) <= a.log_epsrel || err) {
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        nest_set(&a.st->stopped);
      }
      return;
    }
  }
  if constexpr (TAB) {
    // waves 1-3 of the workgroup (one SIMD each; the walkers are wave 0) draw the next
    // generation's table and leave
    if ((int)threadIdx.x >= wl) {
      const int64_t nf = blockDim.x - wl;
      if (a.fuse_retire) {
        // retire the dead points of this workgroup's walkers (see below): element e of the
        // (wl / P) x D block, the scalars with d == 0
        const int64_t w0 = (int64_t)blockIdx.x * (wl / P);
        for (int64_t e = threadIdx.x - wl; e < (wl / P) * D; e += nf) {
          const int64_t wj = w0 + e / D;
          const int d = (int)(e % D);
          if (wj >= a.k) break;
          const int rs = a.key_slot[wj];
          const int64_t m = a.mrep + wj;
          a.dead_x[m * D + d] = a.x[(int64_t)rs * D + d];
          if (d == 0) {
            const double lls = a.ll[rs];
            put_dead(a, m, lls, a.lp[rs]);
            const double lv = a.st->log_vol[gen_par(a)] + a.prefix[wj];
            __hip_atomic_store(a.tv + wj, lls + (lv + a.qadd[wj]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            a.rank[wj] = 0;
          }
        }
        if (a.est_in_walk) {                           // this wave's tv are stored: count it
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if ((threadIdx.x & 63) == 0)
            __hip_atomic_fetch_add(a.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      // (the stride counts the walker workgroups only: a fused launch's merge workgroups fill nothing)
      const int64_t nwb = (int64_t)a.nwalk_blocks;
      walk_draws_fill<!Tgt::kFold>(a, a.mrep + a.k, (int64_t)blockIdx.x * nf + (threadIdx.x - wl), nwb * nf, lt);
#ifdef MCG_NEST_TRACE
      if (a.trace && (int)threadIdx.x == wl && blockIdx.x < 1024)   // the table-filling waves' end
        a.trace[((size_t)0 * 1024 + blockIdx.x) * 8 + 5] = wall_clock64();
#endif
      if constexpr (FM) nest_walk_signal(a);
      return;
    }
  }
  // start: a uniformly random live point satisfying the constraint (nested.ml:63); with k = 1
  // every live point does, so this is Random.int nlive.  Attempt 0 was loaded above.
  const bool first_ok = ll_first >= thr;
  int64_t start = first_ok ? (int64_t)s_first : -1;
  if (!first_ok) {
    for (uint32_t att = 1; att < 4096; ++att) {
      const u32x4 r = rng(wid, att, CALL_START, TAG_NEST_WALK, 0u);
      const uint32_t s = randint(r.x, r.y, n);
      if (a.ll[s] >= thr) {
        start = s;
        break;
      }
    }
  }
  if (start < 0) start = a.key_slot[a.k - 1];
  NT_STAMP(0, 2);
  double cur[NL], y[NL];
  auto load_row_at = [&](double* dst, const double* __restrict__ src) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < Lay::NCL; ++i)
#pragma unroll
      for (int q = 0; q < W; ++q)
        dst[W * i + q] = Lay::valid(sub, i, q) ? src[Lay::dim(sub, i, q)] : 0.0;
  };
  // TAB: the table holds row byte offsets (32-bit: the live set is below 4 GiB); the lane's
  // first dim joins the offset, so a row load is the live set's base (SGPRs) plus one 32-bit
  // VGPR (global_load ... saddr) and one 32-bit add per row
  const char* const xb = (const char*)a.x;
  const uint32_t lane_b = 8u * W * (uint32_t)sub;
  auto load_row_off = [&](double* dst, uint32_t v) __attribute__((always_inline)) {
    const char* src = xb + (v + lane_b);
#pragma unroll
    for (int i = 0; i < Lay::NCL; ++i)
#pragma unroll
      for (int q = 0; q < W; ++q)
        dst[W * i + q] = Lay::valid(sub, i, q) ? *(const double*)(src + 8 * (W * P * i + q)) : 0.0;
  };
  auto refill = [&](double* dst, uint32_t v) __attribute__((always_inline)) {
    if constexpr (TAB) load_row_off(dst, v);
    else load_row_at(dst, a.x + (int64_t)v * D);
  };
  auto load_row = [&](double* dst, int64_t row) __attribute__((always_inline)) {
    const double* __restrict__ src = a.x + row * D;
#pragma unroll
    for (int i = 0; i < Lay::NCL; ++i)
#pragma unroll
      for (int q = 0; q < W; ++q)
        dst[W * i + q] = Lay::valid(sub, i, q) ? src[Lay::dim(sub, i, q)] : 0.0;
  };
  // differential_evolution_proposal's pick_samples (mcmc.ml:199-203): i, then j != i
  auto pick = [&](int64_t s, uint32_t& i, uint32_t& j) __attribute__((always_inline)) {
    const u32x4 ri = rng(wid, (uint32_t)s, CALL_DE_IDX, TAG_NEST_WALK, 0u);
    i = randint(ri.x, ri.y, n);
    const uint32_t jj = randint(ri.z, ri.w, n - 1);
    j = jj + (jj >= i ? 1u : 0u);
  };
  tgt.setup_constraint(thr);
  double cur_l;                                      // mcmc_logl, :54-59
  if (first_ok) {
#pragma unroll
    for (int d = 0; d < NL; ++d) cur[d] = row_first[d];
    cur_l = lp_first;
  } else {
    load_row(cur, start);
    cur_l = (a.ll[start] >= thr) ? a.lp[start] : -__builtin_inf();
  }
  // The random numbers of a group of PD steps are independent of the walker state.  With P = 4
  // lane q of the quad draws those of steps s0 + 4h + q (DE scale, accept uniform, and the DE
  // indices of step s0 + 4h + q + PD, whose rows refill that slot), one group AHEAD: the normal's
  // table gather of group g + 1 is issued before group g's row refills, so waiting for it never
  // drains the prefetched rows (the vector-memory counter is in order).
  struct GroupRng {
    uint32_t pi[PD / 4 > 0 ? PD / 4 : 1], pj[PD / 4 > 0 ? PD / 4 : 1];
    double hop[PD / 4 > 0 ? PD / 4 : 1], lu[PD / 4 > 0 ? PD / 4 : 1];
    NrmPending z[PD / 4 > 0 ? PD / 4 : 1];
  };
  auto group_issue = [&](int64_t s0, GroupRng& G) __attribute__((always_inline)) {
    if constexpr (P == 4 && PD % 4 == 0) {
#pragma unroll
      for (int h = 0; h < PD / 4; ++h) {
        const int64_t sq = s0 + 4 * h + sub;
        const u32x4 rI = rng(wid, (uint32_t)(sq + PD), CALL_DE_IDX, TAG_NEST_WALK, 0u);
        const u32x4 rS = rng(wid, (uint32_t)sq, CALL_DE_SCALE, TAG_NEST_WALK, 0u);
        const u32x4 rA = rng(wid, (uint32_t)sq, CALL_ACCEPT, TAG_NEST_WALK, 0u);
        G.pi[h] = randint(rI.x, rI.y, n);
        const uint32_t pjj = randint(rI.z, rI.w, n - 1);
        G.pj[h] = pjj + (pjj >= G.pi[h] ? 1u : 0u);
        G.z[h] = pnormal_issue(rS.z, nt);
        G.hop[h] = u53(rS.x, rS.y);
        G.lu[h] = plog(u53(rA.x, rA.y), s_lt);
      }
    }
  };
  GroupRng gcur, gnext;
  if constexpr (!TAB) group_issue(0, gcur);   // before the ring's first rows: its gather is then never the newest load
  // TAB: the generation's draws come from the table the previous merge filled (rt_ix, rt_sc),
  // loaded one group ahead like the rows: (scale, log u) of steps s0 + u and the refill indices
  // of steps s0 + PD + u
  unsigned long long tix_next[PD];
  double2 tsc_next[PD];
  // partner rows of steps s .. s + PD - 1 in flight: ring slot u holds step s0 + u
  double bi[PD][NL], bj[PD][NL];
#pragma unroll
  for (int u = 0; u < PD; ++u) {
    uint32_t i0, j0;
    if constexpr (TAB) {
      const unsigned long long ix = tix_ring[u];
      i0 = (uint32_t)ix;
      j0 = (uint32_t)(ix >> 32);
    } else {
      pick(u, i0, j0);
    }
    refill(bi[u], i0);
    refill(bj[u], j0);
  }
  if (!TAB && a.fuse_retire && active) {
    // replace_live_point's retirement (nested.ml:26-43, slot form) of the w-th lowest point: the
    // live set stays frozen during the walk, so its row can go to the dead buffer now -- after
    // the first DE rows are in flight, so that their wait is not queued behind these loads (with
    // the draw table the workgroup's spare waves do this, off the walker's SIMD)
    const int64_t m = a.mrep + w;
    const double* __restrict__ src = a.x + (int64_t)ret_slot * D;
#pragma unroll
    for (int i = 0; i < Lay::NCL; ++i)
#pragma unroll
      for (int q = 0; q < W; ++q)
        if (Lay::valid(sub, i, q)) a.dead_x[m * D + Lay::dim(sub, i, q)] = src[Lay::dim(sub, i, q)];
    if (sub == 0) {
      const double lls = a.ll[ret_slot];
      put_dead(a, m, lls, a.lp[ret_slot]);
      const double lv = a.st->log_vol[gen_par(a)] + a.prefix[w];
      __hip_atomic_store(a.tv + w, lls + (lv + a.qadd[w]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // nested.ml:138-141
      a.rank[w] = 0;
    }
  }
  // whole groups of PD steps with no data-dependent branches around the loads, so the compiler
  // can count the in-flight loads (vmcnt) across iterations; steps past nmcmc only compute
  // 32-bit step counters: gfx950 has no 64-bit scalar less-than, so int64 step tests became a
  // v_mov + v_cmp_lt_i64 pair on the walker's issue-bound wave every step (nmcmc < 2^31: the
  // host caps it)
  const int nm = (int)a.nmcmc;
  NT_STAMP(0, 3);
  // two copies of the loop: with the box test, and without it once the constraint implies it
  // (setup_constraint: box_test is wave-uniform)
  auto walk_loop = [&](auto box_t) __attribute__((always_inline)) {
  constexpr bool kBoxT = decltype(box_t)::value;
  for (int s0 = 0; s0 < nm; s0 += PD) {
    double dsc_g[PD], lu_g[PD];
    uint32_t ip_g[PD], jp_g[PD];
    if constexpr (TAB) {
#pragma unroll
      for (int u = 0; u < PD; ++u) {
        dsc_g[u] = tsc_cur[u].x;
        lu_g[u] = tsc_cur[u].y;
        ip_g[u] = (uint32_t)tix_cur[u];
        jp_g[u] = (uint32_t)(tix_cur[u] >> 32);
      }
#pragma unroll
      for (int u = 0; u < PD; ++u) {                  // the next group's draws go out first
        tsc_next[u] = tsc_lane[tab_off(s0 + PD + u)];
        tix_next[u] = tix_lane[tab_off(s0 + 2 * PD + u)];
      }
    } else if constexpr (P == 4 && PD % 4 == 0) {
      // finish this group's draws and hand step u's values from lane u % 4 to the quad (DPP)
#pragma unroll
      for (int h = 0; h < PD / 4; ++h) {
        const double z0 = pnormal_finish(gcur.z[h]);
        const double dloc = (a.mode_hop != 0.0 && gcur.hop[h] < a.mode_hop) ? 1.0 : a.sigma_de * z0;
        const uint32_t pi = gcur.pi[h], pj = gcur.pj[h];
        const double lloc = gcur.lu[h];
        ip_g[4 * h + 0] = quad_bcast_u32<0>(pi); ip_g[4 * h + 1] = quad_bcast_u32<1>(pi);
        ip_g[4 * h + 2] = quad_bcast_u32<2>(pi); ip_g[4 * h + 3] = quad_bcast_u32<3>(pi);
        jp_g[4 * h + 0] = quad_bcast_u32<0>(pj); jp_g[4 * h + 1] = quad_bcast_u32<1>(pj);
        jp_g[4 * h + 2] = quad_bcast_u32<2>(pj); jp_g[4 * h + 3] = quad_bcast_u32<3>(pj);
        dsc_g[4 * h + 0] = quad_bcast_f64<0>(dloc); dsc_g[4 * h + 1] = quad_bcast_f64<1>(dloc);
        dsc_g[4 * h + 2] = quad_bcast_f64<2>(dloc); dsc_g[4 * h + 3] = quad_bcast_f64<3>(dloc);
        lu_g[4 * h + 0] = quad_bcast_f64<0>(lloc); lu_g[4 * h + 1] = quad_bcast_f64<1>(lloc);
        lu_g[4 * h + 2] = quad_bcast_f64<2>(lloc); lu_g[4 * h + 3] = quad_bcast_f64<3>(lloc);
      }
      group_issue(s0 + PD, gnext);                    // next group's gathers go out first
    } else
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const int64_t s = s0 + u;
      const int64_t sp = s + PD;                       // the step whose rows go into slot u next
      if constexpr (P == 4) {
        // the step's three Philox calls on three lanes of the walker's quad, one call per lane:
        // lane 0 the DE indices of step s + PD (prefetch), lane 1 the DE scale, lane 2 the accept
        // uniform; every lane finishes all three words (same instructions, own data) and the
        // quad broadcasts (DPP) take each value from its lane
        const uint32_t call = sub == 0 ? CALL_DE_IDX : sub == 1 ? CALL_DE_SCALE : CALL_ACCEPT;
        const u32x4 r = rng(wid, (uint32_t)(sub == 0 ? sp : s), call, TAG_NEST_WALK, 0u);
        const uint32_t pi = randint(r.x, r.y, n);
        const uint32_t pjj = randint(r.z, r.w, n - 1);
        const double z0 = pnormal(r.z, nt);
        const double hop_u = u53(r.x, r.y);
        const double dloc = (a.mode_hop != 0.0 && hop_u < a.mode_hop) ? 1.0 : a.sigma_de * z0;
        const double lloc = plog(hop_u, s_lt);
        ip_g[u] = quad_bcast_u32<0>(pi);
        const uint32_t jq = quad_bcast_u32<0>(pjj);
        jp_g[u] = jq + (jq >= ip_g[u] ? 1u : 0u);
        dsc_g[u] = quad_bcast_f64<1>(dloc);
        lu_g[u] = quad_bcast_f64<2>(lloc);
      } else {
        pick(sp, ip_g[u], jp_g[u]);
        const u32x4 rs = rng(wid, (uint32_t)s, CALL_DE_SCALE, TAG_NEST_WALK, 0u);
        if (a.mode_hop != 0.0 && u53(rs.x, rs.y) < a.mode_hop) {
          dsc_g[u] = 1.0;
        } else {
          dsc_g[u] = a.sigma_de * pnormal(rs.z, nt);
        }
        const u32x4 ra = rng(wid, (uint32_t)s, CALL_ACCEPT, TAG_NEST_WALK, 0u);
        lu_g[u] = plog(u53(ra.x, ra.y), s_lt);
      }
    }
    // the serial constrained steps
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const bool live = s0 + u < nm;
#pragma unroll
      for (int d = 0; d < NL; ++d) y[d] = cur[d] + dsc_g[u] * (bj[u][d] - bi[u][d]);
      refill(bi[u], ip_g[u]);                          // refill slot u with step s + PD's rows
      refill(bj[u], jp_g[u]);
      // mcmc.ml:47-48 computes (((ml + 0) - (cur_l + 0)) + 0) - 0 (flat proposal density); the
      // +0 / -0 terms change at most the sign of a zero, so `lu < ratio` is the same test
      if constexpr (Tgt::kFold) {
        // ml is lp_box when the proposal passes and -inf when it fails, and -inf - cur_l fails
        // `lu < ratio` for every cur_l (-inf or NaN), so the step accepts iff it passes and
        // lu < lp_box - cur_l.  That half always holds: cur_l is lp_box (a live point inside the
        // box, or the last accepted proposal) or -inf (a start outside the constraint or on an
        // open box's face), so lp_box - cur_l is +0 or +inf, and log u < 0 for every u53 draw
        // (the largest, 1 - 2^-53, gives -1.1e-16: tests/test_oracle.py).  The step accepts
        // iff it passes: no accept uniform is loaded or compared (the oracle's test, kept
        // literally, takes the same decisions)
        if (tgt.template constraint_box<kBoxT>(y, sub, thr) && live) {
#pragma unroll
          for (int d = 0; d < NL; ++d) cur[d] = y[d];
        }
      } else {
        const bool ok = tgt.constraint(y, sub, a.m, thr);
        const double lpy = tgt.prior(y, sub, a.m);
        const double ml = ok ? lpy : -__builtin_inf();
        const double ratio = ml - cur_l;
        if (live && lu_g[u] < ratio) {
#pragma unroll
          for (int d = 0; d < NL; ++d) cur[d] = y[d];
          cur_l = ml;
        }
      }
    }
    if constexpr (TAB) {
#pragma unroll
      for (int u = 0; u < PD; ++u) {
        tsc_cur[u] = tsc_next[u];
        tix_cur[u] = tix_next[u];
      }
    } else if constexpr (P == 4 && PD % 4 == 0) {
      gcur = gnext;
    }
  }
  };
  if (tgt.box_test) walk_loop(std::true_type{});
  else walk_loop(std::false_type{});
  NT_STAMP(0, 4);
  const double nl = tgt.lik(cur, sub, a.m);
  const double np = tgt.prior(cur, sub, a.m);
  // (FM: the merge role in this launch reads these: stored sc1)
  auto put = [&](auto* p, auto v) __attribute__((always_inline)) {
    if constexpr (FM) wt_store(p, v);
    else *p = v;
  };
  if (active) {
#pragma unroll
    for (int i = 0; i < Lay::NCL; ++i)
#pragma unroll
      for (int q = 0; q < W; ++q)
        if (Lay::valid(sub, i, q)) put(a.nx + w * D + Lay::dim(sub, i, q), cur[W * i + q]);
    if (sub == 0) {
      put(a.nll + w, nl);
      put(a.nlp + w, np);
      if (a.fuse_retire) {                             // the new point's key
        put(a.newk_ll + w, nl);
        put(a.newk_tie + w, -(long long)(a.mrep + w + 1));
        put(a.newk_slot + w, ret_slot);
      }
      if (!(nl >= thr)) nest_set(&a.st->error);      // nested.ml:70-72 -> Failure
    }
  }
  if constexpr (FM) nest_walk_signal(a);
}

// ---- prior draws of the initial live set (nested.ml:126-129, Stats.draw_uniform) ----
template <int D, int LIK>
__global__ void __launch_bounds__(256) nest_init_kernel(const NestArgs a, double* keys_ll,
                                                         long long* keys_tie, int* keys_slot) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n) return;
  const Rng rng{a.k0, a.k1};
  const double* __restrict__ lo = a.m.pri + 2 * D + 1;     // caller's bounds (see mcg_set_prior)
  const double* __restrict__ hi = a.m.pri + 3 * D + 1;     // (DIAG_GAUSS prior: mu, sigma)
  double x[D];
  if (a.m.prior_kind == MCG_PRIOR_DIAG_GAUSS) {
    // Stats.draw_gaussian mu sigma per dim (stats.ml:113-124: mu + sigma z): the normals of dims
    // 4c .. 4c+3 from call c
#pragma unroll
    for (int d = 0; d < D; d += 4) {
      const u32x4 r = rng((uint32_t)s, 0u, (uint32_t)(d >> 2), TAG_NEST_PRIOR, 0u);
      const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (d + j < D) x[d + j] = lo[d + j] + hi[d + j] * pnormal(w[j], kNrmTab);
    }
  } else {
#pragma unroll
    for (int d = 0; d < D; d += 2) {
      const u32x4 r = rng((uint32_t)s, 0u, (uint32_t)(d >> 1), TAG_NEST_PRIOR, 0u);
      x[d] = lo[d] + (hi[d] - lo[d]) * u53(r.x, r.y);
      if (d + 1 < D) x[d + 1] = lo[d + 1] + (hi[d + 1] - lo[d + 1]) * u53(r.z, r.w);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) a.x[s * D + d] = x[d];
  const double l = eval_lik<D, 1, LIK>(x, 0, a.m, a.m.lik);
  a.ll[s] = l;
  a.lp[s] = eval_prior<D, 1>(x, 0, a.m, a.m.pri);
  keys_ll[s] = l;
  keys_tie[s] = s;
  keys_slot[s] = (int)s;
}

hipError_t launch_merge_fused(const NestArgs& a, double* oll, long long* otie, int* oslot, hipStream_t s);

template <int D, int LIK, int P>
hipError_t launch_nest_walk_p(const NestArgs& a, hipStream_t st) {
  // small workgroups: a generation has only k * P lanes, so one wave per workgroup spreads them
  // over all CUs (their LDS tables, L1 and scalar units) instead of packing four per CU
  const int block = kNestWalkBlock;
  const int64_t grid = (a.k * P + block - 1) / block;
  // with the draw table: the same walker waves, each with three table-filling waves beside it
  // (two walker waves and two filling waves per workgroup beyond 256 walker waves)
  NestArgs b = a;
  const int64_t wwaves = (a.k * P + 63) / 64;
  b.walk_waves = wwaves > 256 ? 2 : 1;
  const dim3 gt((unsigned)((wwaves + b.walk_waves - 1) / b.walk_waves)), bt(256);
  constexpr bool kSym = WalkTarget<D, P, LIK>::kReg;   // the |y| <= h form needs the register target
  if (b.fuse_merge && !(b.rt_ix && b.walk_waves == 1 && b.k <= kSmallSort)) {
    // (the fused merge takes one walker wave per workgroup: otherwise walk, then the merge kernel)
    NestArgs c = b;
    c.fuse_merge = 0;
    hipError_t e = launch_nest_walk_p<D, LIK, P>(c, st);
    if (e != hipSuccess) return e;
    return launch_merge_fused(c, c.mrg_ll, c.mrg_tie, c.mrg_slot, st);
  }
  if (b.fuse_merge) {
    // the walk with the generation's merge in the same launch: the merge workgroups after the
    // walkers' (dispatched in order, so every walker workgroup is placed before any of them)
    const int64_t nblk = (a.n - a.k + 255) / 256;
    b.nwalk_blocks = (int32_t)gt.x;
    const dim3 gf((unsigned)(gt.x + nblk + 1));
    if (a.m.prior_kind == MCG_PRIOR_DIAG_GAUSS)
      hipLaunchKernelGGL((nest_walk_kernel<D, LIK, P, true, false, true, true>), gf, bt, 0, st, b);
    else if (kSym && b.sym_box)
      hipLaunchKernelGGL((nest_walk_kernel<D, LIK, P, true, kSym, false, true>), gf, bt, 0, st, b);
    else
      hipLaunchKernelGGL((nest_walk_kernel<D, LIK, P, true, false, false, true>), gf, bt, 0, st, b);
    return hipGetLastError();
  }
  // TAB: the previous generation's merge tail (split merge) in tl_nblk workgroups past the walkers'
  b.nwalk_blocks = (int32_t)gt.x;
  const dim3 gts((unsigned)(gt.x + (b.split ? b.tl_nblk : 0) + (b.est_in_walk ? 1 : 0)));
  if (a.m.prior_kind == MCG_PRIOR_DIAG_GAUSS) {
    if (b.rt_ix) hipLaunchKernelGGL((nest_walk_kernel<D, LIK, P, true, false, true>), gts, bt, 0, st, b);
    else hipLaunchKernelGGL((nest_walk_kernel<D, LIK, P, false, false, true>), dim3((unsigned)grid), dim3(block), 0, st, a);
    return hipGetLastError();
  }
  if (b.rt_ix && kSym && b.sym_box) hipLaunchKernelGGL((nest_walk_kernel<D, LIK, P, true, kSym>), gts, bt, 0, st, b);
  else if (b.rt_ix) hipLaunchKernelGGL((nest_walk_kernel<D, LIK, P, true, false>), gts, bt, 0, st, b);
  else hipLaunchKernelGGL((nest_walk_kernel<D, LIK, P, false, false>), dim3((unsigned)grid), dim3(block), 0, st, a);
  return hipGetLastError();
}

template <int D, int LIK>
hipError_t launch_nest_walk(const NestArgs& a, hipStream_t st) {
  // lanes per walker: the separable likelihoods split the dims over several lanes, which gives
  // the few-thousand-walker generations that many times the lanes and shortens each walker's
  // serial step (fewer dims per lane).  One 4-dim block per lane on 8 lanes when D % 32 == 0
  // (the bench's D = 32 leg: nested run 0.125 -> 0.103 s, A/B on one box), else 4 (D % 16 == 0)
  // or 2 (D % 8 == 0) lanes; MCG_NEST_LANES: "narrow" (4 at D % 32 == 0), "wide" (two dims per
  // lane at D = 8 / 16: 4 / 8 lanes), or the lane count
  constexpr bool sep = LIK == MCG_LIK_DIAG_GAUSS || LIK == MCG_LIK_GAUSS_SHELL || LIK == MCG_LIK_FLAT;
  constexpr int P = (sep && D % 16 == 0) ? 4 : (sep && D % 8 == 0) ? 2 : 1;
  if constexpr (sep && D % 32 == 0) {
    if (a.lanes_hint != -2 && a.lanes_hint != 4) return launch_nest_walk_p<D, LIK, 8>(a, st);
  }
  if constexpr (sep && (D == 16 || D == 8)) {          // two dims per lane (WalkLayout W = 2)
    if (a.lanes_hint == 2 * P || a.lanes_hint == -1) return launch_nest_walk_p<D, LIK, 2 * P>(a, st);
    // D 16 beyond 256 walker waves (k > 4,096): 8 lanes of 2 dims put a walker wave on every
    // SIMD (k 8,192: walk 38.0 -> 35.0 us a generation, same box; at k 4,096 the 4-lane split
    // stays ahead, 23.7 vs 29.1 us, profiles/r05/lanes)
    if constexpr (D == 16) {
      if (a.lanes_hint == 0 && a.k * P > 256 * 64) return launch_nest_walk_p<D, LIK, 2 * P>(a, st);
    }
  }
  return launch_nest_walk_p<D, LIK, P>(a, st);
}

template <int D, int LIK>
hipError_t launch_nest_init(const NestArgs& a, double* kl, long long* kt, int* ks, hipStream_t st) {
  const int64_t grid = (a.n + 255) / 256;
  hipLaunchKernelGGL((nest_init_kernel<D, LIK>), dim3((unsigned)grid), dim3(256), 0, st, a, kl, kt, ks);
  return hipGetLastError();
}

// generic kernels (mcg_nested_kernels.hip)
hipError_t launch_sort_keys(double* ll, long long* tie, int* slot, double* tll, long long* ttie,
                            int* tslot, int64_t n, bool* result_in_tmp, hipStream_t st,
                            const NestDevState* stop);
hipError_t launch_merge_new(const NestArgs& a, double* out_ll, long long* out_tie, int* out_slot,
                            const double* new_ll, const long long* new_tie, const int* new_slot,
                            hipStream_t st);
// the final live rows in key order behind the dead rows
hipError_t launch_gather_live(const double* x, const double* ll, const double* lp, const int* slot, int64_t n,
                              int D, double* ox, double* oll, double* olp, hipStream_t st);
// the run's rows (x | ll | lp) into a device buffer of row stride `stride` (mcg_nested_rows_into)
hipError_t launch_nested_rows(const double* x, int Dk, int D, const double* ll, const double* lp, int64_t n,
                              double* out, int64_t stride, int pts, hipStream_t st);
// the walkers' draws of the generation starting at replacement mrep (the first generation's table)
hipError_t launch_walk_draws(const NestArgs& a, int64_t mrep, hipStream_t st);
hipError_t launch_check_sorted(const double* ll, const long long* tie, int64_t n, long long gen,
                               long long* out, hipStream_t st);
// retire the k lowest; the last workgroup also folds the generation into the running estimate
hipError_t launch_retire(const NestArgs& a, int D, hipStream_t st);
// every kKeySample-th of n sorted keys (indices kKeySample-1, 2 kKeySample-1, ...) into s*
hipError_t launch_key_sample(const double* ll, const long long* tie, int64_t n, double* sll,
                             long long* stie, hipStream_t st, NestDevState* state = nullptr);
// k <= 4096: the generation's unsorted new keys merged into the survivors in one launch (plus the
// estimate and the slot writes): keys -> o*
hipError_t launch_merge_fused(const NestArgs& a, double* oll, long long* otie, int* oslot, hipStream_t s);
// split merge (k <= 4096): the head (merged keys [0, k), estimate, L_max, the new points' slot
// writes) and a stand-alone tail (the last generation's positions >= k, when no walk ran it)
hipError_t launch_merge_head(const NestArgs& a, double* oll, long long* otie, int* oslot, hipStream_t s);
hipError_t launch_merge_tail(const NestArgs& a, hipStream_t s);
// k <= 4096: new keys sorted into o* by counting ranks (a.rank zeroed by the retire kernel)
hipError_t launch_sort_new_small(const NestArgs& a, double* oll, long long* otie, int* oslot,
                                 hipStream_t st);

typedef hipError_t (*nest_walk_fn)(const NestArgs&, hipStream_t);
typedef hipError_t (*nest_init_fn)(const NestArgs&, double*, long long*, int*, hipStream_t);
nest_walk_fn find_nest_walk(int D, int lik);
nest_init_fn find_nest_init(int D, int lik);

}  // namespace mcg
