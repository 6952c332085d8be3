// mcg_mh_kernel.h -- the batched Metropolis-Hastings kernel.
//
// Restates Mcmc.make_mcmc_sampler (mcmc.ml:37-56) driven by Mcmc.mcmc_array (mcmc.ml:58-72)
// for N independent chains.  Layout and execution (DESIGN.md §MH kernel):
//   * P lanes per chain (P in {1,2,4,8}); lane `sub` owns the dims of Philox calls
//     c = sub, sub+P, ... (4 dims per call); chain state stays in VGPRs for the whole launch;
//   * SoA state x[d][chain] in HBM is read once and written once per launch (coalesced);
//   * one Philox4x32-10 call gives 4 proposal normals (one quantile-table normal per word);
//   * the log-target is a canonical 8-accumulator sum (reduction tree fixed, P-independent);
//   * the accept test `log u < ratio` (mcmc.ml:49) is packed per step into a 64-lane
//     wavefront ballot -> accept bitmap row;
//   * recorded samples optionally fold into per-chain Welford moments and log-space
//     harmonic-mean partials (Evidence.evidence_harmonic_mean, evidence.ml:101-107).
#pragma once
#include "mcg_device.h"
#include "mcg_math.h"
#include "mcg.h"
#include <utility>

namespace mcg {

// Lane layout of a chain on P lanes: lane `sub` owns the W-dim blocks c = sub, sub + P, ... (dims
// W c .. W c + W - 1).  W = 4: the blocks are the Philox calls of the Gaussian proposal's normals
// (dims 4c .. 4c+3 from call c).  W = 2 (D = 2P, the kD independence proposal only): a lane owns
// two dims, whose box-draw uniforms are exactly one Philox call (dims 2c, 2c + 1 from call c), and
// the two lanes of a canonical accumulator chain their fmas in dim order (reduce_canon_w2).
template <int D, int P, int W = 4>
struct Layout {
  static_assert(P == 1 || P == 2 || P == 4 || P == 8, "P must divide 8");
  static_assert(W == 4 || (W == 2 && P >= 2 && D == 2 * P), "W = 2: two dims per lane, D = 2P");
  static constexpr int NC = (D + W - 1) / W;             // blocks per chain
  static constexpr int NCL = (NC + P - 1) / P;           // blocks owned by one lane
  static constexpr int NL = NCL * W;                     // local dims
  static constexpr int NA = W == 2 ? 1 : 8 / P;          // local accumulators
  static_assert(P == 1 || D % (W * P) == 0, "P > 1 needs D % WP == 0");
  __device__ static __forceinline__ int dim(int sub, int i, int q) { return W * (sub + P * i) + q; }
  __device__ static __forceinline__ bool valid(int sub, int i, int q) {
    return q < W && (P > 1 || (W * i + q) < D);
  }
};

// f(integral_constant<int, 0>) .. f(integral_constant<int, N - 1>), in order (compile-time slots)
template <int N, class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}

// steps of kD draw prefetch on P > 1 lanes (mh_kernel's KDA)
#ifndef MCG_KD_AHEAD
#define MCG_KD_AHEAD 4
#endif
constexpr int kKdAhead = MCG_KD_AHEAD;
// non-kD steps on P > 1 lanes unrolled by P (MCG_STEP_UNROLL=1)
#ifndef MCG_STEP_UNROLL
#define MCG_STEP_UNROLL 0
#endif
constexpr bool kStepUnroll = MCG_STEP_UNROLL != 0;

// the width of a chain's lane blocks: two dims per lane where the kD proposal runs on D = 2P lanes
template <int D, int P, int PROP>
constexpr int lane_width() {
  return (PROP == MCG_PROP_KD_INTERP && P >= 2 && D == 2 * P) ? 2 : 4;
}

// The canonical sum for W = 2 (D = 2P): lane sub holds the terms of dims 2 sub, 2 sub + 1, which
// belong to accumulator A_j, j = sub / 2.  The even lane of the pair folds dims 4j, 4j + 1 from
// zero, the odd lane continues from that partial with dims 4j + 2, 4j + 3 (the sequential fma
// chain of A_j), and the odd lanes (A_0 .. A_{P/2-1}) meet in the canonical tree
// ((A0 + A4) + (A2 + A6)) + ((A1 + A5) + (A3 + A7)), whose A_{P/2} .. A_7 are zero here (x + 0 = x
// for the sums of squares): (A0 + A2) + (A1 + A3) at P = 8, A0 + A1 at P = 4, A0 at P = 2.  Even
// lanes take their odd neighbour's value.  Additions are commutative, so every lane of the tree
// holds the same bits.
template <int P>
__device__ __forceinline__ double reduce_canon_w2(double e0, double e1, int sub) {
  static_assert(P == 2 || P == 4 || P == 8, "W = 2 chains run on 2, 4 or 8 lanes");
  const double t = fma(e1, e1, fma(e0, e0, 0.0));
  const double tp = xor_lane_d<1>(t);
  const double a = fma(e1, e1, fma(e0, e0, tp));
  double c;
  if constexpr (P == 8) {
    const double b = a + xor_lane_d<4>(a);
    c = b + xor_lane_d<2>(b);
  } else if constexpr (P == 4) {
    c = a + xor_lane_d<2>(a);
  } else {
    c = a;
  }
  const double o = xor_lane_d<1>(c);
  return (sub & 1) ? c : o;
}

// reduce the lane-local accumulators of the canonical tree across the P lanes of a chain
template <int P>
__device__ __forceinline__ double reduce_canon(const double* a) {
  if constexpr (P == 1) {
    return canon8(a);
  } else if constexpr (P == 2) {
    double c = (a[0] + a[2]) + (a[1] + a[3]);
    return c + xor_lane_d<1>(c);
  } else if constexpr (P == 4) {
    double b = a[0] + a[1];
    double c = b + xor_lane_d<2>(b);
    return c + xor_lane_d<1>(c);
  } else {
    double b = a[0] + xor_lane_d<4>(a[0]);
    double c = b + xor_lane_d<2>(b);
    return c + xor_lane_d<1>(c);
  }
}

template <int P>
__device__ __forceinline__ int and_lanes(int v) {
  if constexpr (P >= 8) v &= xor_lane_i<4>(v);
  if constexpr (P >= 4) v &= xor_lane_i<2>(v);
  if constexpr (P >= 2) v &= xor_lane_i<1>(v);
  return v;
}

// gather bit (c*P) of a 64-lane ballot for c in [0, 64/P)
template <int P>
__device__ __forceinline__ uint64_t compress_ballot(uint64_t m) {
  if constexpr (P == 1) {
    return m;
  } else if constexpr (P == 2) {
    m &= 0x5555555555555555ull;
    m = (m | (m >> 1)) & 0x3333333333333333ull;
    m = (m | (m >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    m = (m | (m >> 4)) & 0x00FF00FF00FF00FFull;
    m = (m | (m >> 8)) & 0x0000FFFF0000FFFFull;
    m = (m | (m >> 16)) & 0x00000000FFFFFFFFull;
    return m;
  } else if constexpr (P == 4) {
    m &= 0x1111111111111111ull;
    m = (m | (m >> 3)) & 0x0303030303030303ull;
    m = (m | (m >> 6)) & 0x000F000F000F000Full;
    m = (m | (m >> 12)) & 0x000000FF000000FFull;
    m = (m | (m >> 24)) & 0x000000000000FFFFull;
    return m;
  } else {
    m &= 0x0101010101010101ull;
    m = (m | (m >> 7)) & 0x0003000300030003ull;
    m = (m | (m >> 14)) & 0x0000000F0000000Full;
    m = (m | (m >> 28)) & 0x00000000000000FFull;
    return m;
  }
}

// kD descent (Interpolate_pdf.find_cell, interpolate_pdf.ml:101-109): go left iff the point
// is in the left child's inclusive box; boxes nest, so outside the root box -> always right.
template <int D>
__device__ __forceinline__ int kd_find_leaf(const KdNode* __restrict__ nodes,
                                            const double* __restrict__ root, const double* v) {
  // (branch-free: every root bound load in flight together)
  bool inside = true;
#pragma unroll
  for (int d = 0; d < D; ++d) inside = inside & (v[d] >= root[d]) & (v[d] <= root[D + d]);
  int node = 0;
  for (int guard = 0; guard < 4096; ++guard) {
    KdNode nd = nodes[node];
    if (nd.dim < 0) return -1 - nd.dim;
    // the split coordinate by a select chain kept opaque: folded back into v[nd.dim], it put v
    // on the scratch stack, and the scratch stores pending at the caller's join forced vmcnt(0)
    // (loads and stores pending together) on the MH step's main path
    double c = v[0];
#pragma unroll
    for (int d = 1; d < D; ++d) {
      c = (nd.dim == d) ? v[d] : c;
      asm volatile("" : "+v"(c));
    }
    bool left = inside && (c <= nd.split);
    node = left ? node + 1 : nd.right;
  }
  return 0;
}

// Mcmc.uniform_wrapping (mcmc.ml:187-196): the reference's reflection loop, operation for
// operation, for up to kWrapExact reflections (|dx| up to ~2048 box widths: every practical
// step).  Two inputs on which the reference's loop never ends get an exit: a point that lands
// exactly on xmax (the reflection maps xmax to itself: returned as is), and one so far out that
// reflections stop shrinking it (|nx| >> width, where rounding makes a 2-cycle).  Past
// kWrapExact reflections the remaining excess is folded in one step by the loop's
// real-arithmetic limit, a triangle wave of period 2 (xmax - xmin) (fmod is exact).  Shared
// with the oracle (oracle.c wrap_uniform) bit for bit.
constexpr int kWrapExact = 1024;
__device__ __forceinline__ double wrap_uniform(double xmin, double xmax, double dx, double x,
                                               double u) {
  double nx = x + (u - 0.5) * dx;
  for (int it = 0; it < kWrapExact; ++it) {
    if (nx < xmin) {
      nx = xmin + (xmin - nx);
    } else if (nx >= xmax) {
      const double r = xmax - (nx - xmax);
      if (r == nx) return nx;
      nx = r;
    } else {
      return nx;
    }
  }
  const double w = xmax - xmin;
  double m = fmod(nx - xmin, 2.0 * w);
  if (m < 0.0) m += 2.0 * w;
  return m < w ? xmin + m : xmax - (m - w);
}

// ---- Mcmc.combine_jump_proposals (mcmc.ml:165-185), device layout from mcg_runtime.cpp
// pack_mixture: [ncomp], then per component (stride 5 + 3D) p, log p, kind, ljp mode, C, params.
template <int D>
struct MixLayout {
  static constexpr int kStride = 5 + 3 * D;
  __device__ static __forceinline__ const double* comp(const double* q, int c) { return q + 1 + c * kStride; }
};

// the reference's private log-sum (mcmc.ml:155-163): log (1 + exp), not log1p
__device__ __forceinline__ double lse_mix(double la, double lb, const double2* lt) {
  if (la == -__builtin_inf() && lb == -__builtin_inf()) return -__builtin_inf();
  if (la > lb) return la + plog(1.0 + pexp(lb - la), lt);
  return lb + plog(1.0 + pexp(la - lb), lt);
}

// log_jump_prob of the mixture from `from` to `to`: fold over the components of
// log p_i + ljp_i from to (mcmc.ml:175-182); lq_to = log q(to) of the kD tree (if any)
template <int D>
__device__ __forceinline__ double mix_log_jp(const double* __restrict__ q, const double* from,
                                             const double* to, double lq_to, const double2* lt) {
  using M = MixLayout<D>;
  const int nc = (int)q[0];
  double acc = -__builtin_inf();
  for (int c = 0; c < nc; ++c) {
    const double* m = M::comp(q, c);
    const int kind = (int)m[2];
    double lj = 0.0;
    if (m[3] != 0.0) {
      if (kind == MCG_MIX_GAUSS) {
        double S = 0.0;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          const double e = (to[d] - from[d]) * m[5 + D + d];
          S = fma(e, e, S);
        }
        lj = m[4] - 0.5 * S;
      } else if (kind == MCG_MIX_SHIFT_UNIFORM) {
        bool in = true;
#pragma unroll
        for (int d = 0; d < D; ++d) in = in && (to[d] >= from[d] + m[5 + d]) && (to[d] <= from[d] + m[5 + D + d]);
        lj = in ? m[4] : -__builtin_inf();
      } else {
        lj = lq_to;                                      // KD_INTERP: log jump_prob to
      }
    }
    acc = lse_mix(acc, m[1] + lj, lt);
  }
  return acc;
}

__device__ __forceinline__ bool mix_has_kd(const double* __restrict__ q, int stride) {
  const int nc = (int)q[0];
  bool kd = false;
  for (int c = 0; c < nc; ++c) kd = kd || ((int)q[1 + c * stride + 2] == MCG_MIX_KD_INTERP);
  return kd;
}

// The Welford weight 1/(R+1) of record R (host IEEE division, MhArgs::inv_n): R is the same for
// every lane, so this is a scalar load (lgkmcnt).  As a vector load, the step that copied it into
// the next record's weight register waited with vmcnt(0), which also drained every load issued
// ahead (the kD proposal's leaf and box prefetches: C4 stalled there once per step).
__device__ __forceinline__ double welford_weight(const MhArgs& a, int64_t idx) {
  typedef const __attribute__((address_space(4))) double kdouble;
  return ((kdouble*)a.inv_n)[idx];
}

// Q: a generic pointer, or (the MH kernel's per-step evaluation) a constant-address-space one,
// whose uniform loads become scalar loads (the scalar cache and lgkmcnt, not vmcnt: a per-step
// vector load of the constants waited with vmcnt(0) and drained every load issued ahead)
template <int D, int P, int LIK, typename Q = const double* __restrict__, int W = 4>
__device__ __forceinline__ double eval_lik(const double* y, int sub, const MhArgs& a, Q q) {
  using L = Layout<D, P, W>;
  if constexpr (LIK == MCG_LIK_FLAT) {
    return 0.0;
  } else if constexpr ((LIK == MCG_LIK_DIAG_GAUSS || LIK == MCG_LIK_GAUSS_SHELL) && W == 2) {
    // two dims per lane (dims 2 sub, 2 sub + 1): the pair-chained canonical accumulator
    double e[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int d = L::dim(sub, 0, k);
      e[k] = LIK == MCG_LIK_DIAG_GAUSS ? fma(y[k], q[D + d], -q[d]) : y[k] - q[d];
    }
    const double S = reduce_canon_w2<P>(e[0], e[1], sub);
    if constexpr (LIK == MCG_LIK_DIAG_GAUSS) {
      return q[2 * D] - 0.5 * S;
    } else {
      const double r = psqrt(S);
      const double qq = (r - q[D]) * q[D + 1];
      return q[D + 2] - 0.5 * qq * qq;
    }
  } else if constexpr (LIK == MCG_LIK_DIAG_GAUSS || LIK == MCG_LIK_GAUSS_SHELL) {
    // DIAG: q = mu/sigma[D], 1/sigma[D], C        SHELL: q = c[D], R, iw, C
    double A[L::NA];
#pragma unroll
    for (int j = 0; j < L::NA; ++j) A[j] = 0.0;
#pragma unroll
    for (int i = 0; i < L::NCL; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!L::valid(sub, i, k)) continue;
        int d = L::dim(sub, i, k);
        double e;
        if constexpr (LIK == MCG_LIK_DIAG_GAUSS) e = fma(y[4 * i + k], q[D + d], -q[d]);
        else e = y[4 * i + k] - q[d];
        A[i % L::NA] = fma(e, e, A[i % L::NA]);
      }
    double S = reduce_canon<P>(A);
    if constexpr (LIK == MCG_LIK_DIAG_GAUSS) {
      return q[2 * D] - 0.5 * S;
    } else {
      double r = psqrt(S);
      double qq = (r - q[D]) * q[D + 1];
      return q[D + 2] - 0.5 * qq * qq;
    }
  } else if constexpr (LIK == MCG_LIK_FULLCOV_GAUSS) {
    static_assert(P == 1 && W == 4, "FULLCOV: one lane per chain");
    // q = mu[D], C, U[D*D]
    double r[D];
#pragma unroll
    for (int d = 0; d < D; ++d) r[d] = y[d] - q[d];
    double A[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) A[j] = 0.0;
    const auto U = q + D + 1;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double t = 0.0;
#pragma unroll
      for (int j = i; j < D; ++j) t = fma(U[i * D + j], r[j], t);
      const int k = (i & 3) | (((i >> 4) & 1) << 2);   // FULLCOV accumulator (mcg_fullcov_kernel.h)
      A[k] = fma(t, t, A[k]);
    }
    return q[D] - 0.5 * canon8(A);
  } else if constexpr (LIK == MCG_LIK_GAUSS_MIX) {
    static_assert(W == 4, "GAUSS_MIX: four-dim lane blocks");
    // log (sum_i exp g_i) over a.data_n components (test/nested_test.ml:52-57), g_i the DIAG
    // canonical form of component i (q + i (2D + 1): mu/sigma[D], 1/sigma[D], C_i), folded by a
    // one-pass max-shifted log-sum-exp in component order: s = sum_i exp(g_i - M) with the
    // running max M rescaling s when it moves (the reference's exp overflows above g = 709)
    double M = -__builtin_inf(), s = 0.0;
    const int nc = (int)a.data_n;
    for (int c = 0; c < nc; ++c) {
      const auto qc = q + c * (2 * D + 1);
      double A[L::NA];
#pragma unroll
      for (int j = 0; j < L::NA; ++j) A[j] = 0.0;
#pragma unroll
      for (int i = 0; i < L::NCL; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!L::valid(sub, i, k)) continue;
          const int d = L::dim(sub, i, k);
          const double e = fma(y[4 * i + k], qc[D + d], -qc[d]);
          A[i % L::NA] = fma(e, e, A[i % L::NA]);
        }
      const double g = qc[2 * D] - 0.5 * reduce_canon<P>(A);
      if (g > M) {
        s = s * pexp(M - g) + 1.0;
        M = g;
      } else {
        s = s + pexp(g - M);
      }
    }
    return M == -__builtin_inf() ? M : M + plog(s);
  } else {
    // GAUSS_DATA / CAUCHY_DATA (bin/gaussian_cauchy.ml:149-164), D = 2 nd, y = (mu, sigma)
    static_assert(P == 1 && W == 4, "DATA: one lane per chain");
    constexpr int ND = D / 2;
    const double PI = 3.14159265358979323846;
    double lterm[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) lterm[j] = a.is_cauchy ? plog(PI * y[ND + j]) : plog(y[ND + j]);
    double acc = 0.0;
    for (int64_t i = 0; i < a.data_n; ++i) {
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        double dx = (q[i * ND + j] - y[j]) / y[ND + j];
        double term;
        if (a.is_cauchy) term = (0.0 - lterm[j]) - plog(1.0 + dx * dx);
        else term = (-0.91893853320467274178 - lterm[j]) - 0.5 * dx * dx;
        acc = acc + term;
      }
    }
    return acc + 0.0;
  }
}

// MCG_PRIOR_DIAG_GAUSS: Stats.log_multi_gaussian mu sigma y (stats.ml:98-108) in the canonical
// form of the DIAG_GAUSS likelihood -- its device constants [mu/sigma[D], 1/sigma[D], C] head the
// prior descriptor (mcg_runtime.cpp pack_prior), so the same code evaluates it bit for bit
template <int D, int P, typename Q = const double* __restrict__, int W = 4>
__device__ __forceinline__ double eval_gauss_prior(const double* y, int sub, const MhArgs& a, Q q) {
  return eval_lik<D, P, MCG_LIK_DIAG_GAUSS, Q, W>(y, sub, a, q);
}

template <int D, int P, typename Q = const double* __restrict__, int W = 4>
__device__ __forceinline__ double eval_prior(const double* y, int sub, const MhArgs& a, Q q) {
  using L = Layout<D, P, W>;
  if (a.prior_kind == MCG_PRIOR_FLAT) return 0.0;
  if (a.prior_kind == MCG_PRIOR_DIAG_GAUSS) return eval_gauss_prior<D, P, Q, W>(y, sub, a, q);
  int inb = 1;
  if (a.ubox) {
    // one box for every dim: the bounds are kernel arguments (SGPRs).  Per-dim loads of the
    // bounds were compiled into a chain of branches, one global load and a full vmcnt wait each
    // (the kD kernel of C4 spent most of its step there)
#pragma unroll
    for (int i = 0; i < L::NCL; ++i)
#pragma unroll
      for (int k = 0; k < W; ++k) {
        if (!L::valid(sub, i, k)) continue;
        const double v = y[W * i + k];
        inb &= (int)(v >= a.box_lo) & (int)(v <= a.box_hi);
      }
  } else {
    // all bounds loaded before any compare (the same predicate, no per-dim wait)
    double lo[L::NL], hi[L::NL];
#pragma unroll
    for (int i = 0; i < L::NCL; ++i)
#pragma unroll
      for (int k = 0; k < W; ++k) {
        const int d = L::valid(sub, i, k) ? L::dim(sub, i, k) : 0;
        lo[W * i + k] = q[d];
        hi[W * i + k] = q[D + d];
      }
#pragma unroll
    for (int i = 0; i < L::NCL; ++i)
#pragma unroll
      for (int k = 0; k < W; ++k) {
        if (!L::valid(sub, i, k)) continue;
        const double v = y[W * i + k];
        inb &= (int)(v >= lo[W * i + k]) & (int)(v <= hi[W * i + k]);   // closed form of the box (see above)
      }
  }
  inb = and_lanes<P>(inb);
  return inb ? q[2 * D] : -__builtin_inf();
}

constexpr int kUniGaussPrior = 3;

// the fused step (per Philox call: normals, coordinates, likelihood terms, box test) applies to
// separable likelihoods with a Gaussian random-walk proposal
template <int LIK, int PROP>
constexpr bool separable() {
  return (LIK == MCG_LIK_DIAG_GAUSS || LIK == MCG_LIK_GAUSS_SHELL || LIK == MCG_LIK_FLAT) &&
         PROP == MCG_PROP_GAUSS;
}

template <int D, int P, int W = 4>
struct AccumCfg {
  // Welford accumulators of the lane's NL dims: in VGPRs when NL <= 8, else in LDS ([NL][256]
  // doubles each, conflict-free) when they fit in 64 KiB per block, else read-modified-written in
  // HBM at each record.
  static constexpr bool kReg = Layout<D, P, W>::NL <= 8;
  static constexpr bool kLds = !kReg && Layout<D, P, W>::NL <= 16;
  static constexpr int kLdsBytes = kLds ? 2 * Layout<D, P, W>::NL * 256 * 8 : 0;
};

// Waves per SIMD the kernel is built for.  The fused Gaussian step with at most 8 dims per lane
// (C2: D 32 on 4 lanes) fits 168 registers -- three waves per SIMD -- when its normals are
// evaluated one at a time, each normal's two table rows gathered one normal ahead (kPipe; batched
// gathers' 32 in-flight registers would spill): C2 1.87e10 -> 1.96e10 MH steps/s against two
// waves with batched gathers.  Everything else is left to the compiler's register budget, its
// four normals of a Philox call gathered together (one LDS wait).
template <int D, int P, int LIK, int PROP, int UNI = 0>
struct MhShape {
  static constexpr bool kThree = separable<LIK, PROP>() && UNI != kUniGaussPrior &&
                                 Layout<D, P, lane_width<D, P, PROP>()>::NL <= 8;
  static constexpr bool kPipe = kThree;
  // (one lane per chain, D <= 8: the whole chain per lane does not fit 168 registers; those
  // instances are built for the two waves per SIMD they reach)
  static constexpr int kWaves = kThree ? (P > 1 ? 3 : 2) : 1;
  static constexpr int kBlock = 256;
  static constexpr bool kBatchNormals = !kThree;
  // harmonic-mean partials in LDS only where that was measured (C2: P = 4, three waves); a P = 1
  // instance would hold 2 x 8 x 256 doubles (32 KB) of LDS per workgroup for them, halving the
  // workgroups per CU of the small-D kD / mixture / generic kernels, so those keep them in VGPRs
  static constexpr bool kHmLds = P >= 4 || kThree;
};

// UNI: 0 = constants through pointers; 1 = isotropic proposal scale and one box [lo, hi] for
// every dim as kernel arguments; 2 = the same with a symmetric box [-h, h], tested as |y| <= h
// (one compare per dim; the same predicate as lo <= y <= hi for every double, NaN included);
// kUniGaussPrior = a separable likelihood under a DIAG_GAUSS prior: the step is not fused (the
// fused step folds a box test, not a second canonical sum), it runs the generic proposal +
// eval_lik + eval_prior path
template <int D, int P, int LIK, int PROP, int UNI>
__global__ void __launch_bounds__((MhShape<D, P, LIK, PROP, UNI>::kBlock), (MhShape<D, P, LIK, PROP, UNI>::kWaves)) mh_kernel(const MhArgs a) {
  using Shape = MhShape<D, P, LIK, PROP, UNI>;
  constexpr int kBlk = Shape::kBlock;
  constexpr int kW = lane_width<D, P, PROP>();
  using L = Layout<D, P, kW>;
  using ACfg = AccumCfg<D, P, kW>;
  constexpr bool kSeparable = separable<LIK, PROP>() && UNI != kUniGaussPrior;
  static_assert(kSeparable || UNI == 0 || (UNI == kUniGaussPrior && separable<LIK, PROP>()),
                "UNI applies to the fused separable step");
  static_assert(!kSeparable || kW == 4, "the fused Gaussian step takes four-dim lane blocks");
  extern __shared__ double lds_acc[];
  __shared__ double2 s_lt[kLogTabN];                 // math tables staged in LDS (gathers)
  __shared__ double2 s_nt[kNrmTabN];
  for (int i = threadIdx.x; i < kLogTabN; i += blockDim.x) s_lt[i] = kLogTab[i];
  for (int i = threadIdx.x; i < kNrmTabN; i += blockDim.x) s_nt[i] = kNrmTab[i];
  __syncthreads();
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int sub = (int)(tid & (P - 1));
  const int64_t chain = tid / P;
  const bool active = chain < a.N;
  const int64_t c = active ? chain : 0;
  const int64_t N = a.N;
  const Rng rng{a.k0, a.k1};
  const uint32_t gid = a.chain_offset + (uint32_t)c;
  const int lane = threadIdx.x & 63;

  double x[L::NL], y[L::NL];
#pragma unroll
  for (int i = 0; i < L::NCL; ++i)
#pragma unroll
    for (int k = 0; k < kW; ++k)
      x[kW * i + k] = L::valid(sub, i, k) ? a.x[(int64_t)L::dim(sub, i, k) * N + c] : 0.0;
  double ll = a.ll[c], lp = a.lp[c];
  double lq = 0.0;
  if constexpr (PROP == MCG_PROP_KD_INTERP) {
    if constexpr (P == 1) {
      lq = a.kd_logq[kd_find_leaf<D>(a.kd_nodes, a.kd_root, x)];
    } else {
      // the descent needs every dim: the chain's whole start point, read once per launch
      double xf[D];
#pragma unroll
      for (int d = 0; d < D; ++d) xf[d] = a.x[(int64_t)d * N + c];
      lq = a.kd_logq[kd_find_leaf<D>(a.kd_nodes, a.kd_root, xf)];
    }
  }
  bool mix_kd = false;
  if constexpr (PROP == MCG_PROP_MIXTURE) {
    mix_kd = mix_has_kd(a.prop, MixLayout<D>::kStride);
    if (mix_kd) lq = a.kd_logq[kd_find_leaf<D>(a.kd_nodes, a.kd_root, x)];
  }
  unsigned long long na = 0;

  const bool accum = (a.flags & RUNF_ACCUMULATE) != 0;
  // harmonic-mean partials of the 8 record classes R & 7: lane `sub` owns the
  // classes c = sub + P l.  The -ll of record R is parked in lane R mod P and folded when the
  // group of P records is complete, so each lane evaluates one exp per P records.
  constexpr int NH = P >= 8 ? 1 : 8 / P;
  // the partials live in LDS ([2 NH][256], conflict-free): touched once per P records, they
  // would otherwise hold 4 NH VGPRs through the whole step
  constexpr bool kHmLds = Shape::kHmLds;
  __shared__ double s_hm[kHmLds ? 2 * NH * kBlk : 1];
  double hcm_r[kHmLds ? 1 : NH], hcs_r[kHmLds ? 1 : NH];
  auto hcm = [&](int l) -> double& {
    if constexpr (kHmLds) return s_hm[(2 * l) * kBlk + threadIdx.x];
    else return hcm_r[l];
  };
  auto hcs = [&](int l) -> double& {
    if constexpr (kHmLds) return s_hm[(2 * l + 1) * kBlk + threadIdx.x];
    else return hcs_r[l];
  };
  double hm_pv = 0.0;
  bool hm_pok = false;
  // accumulator slot j of this lane: VGPR, LDS [j][threadIdx] or HBM [dim][chain]
  constexpr int NR = ACfg::kReg ? L::NL : 1;
  double rmean[NR], rm2[NR];
  auto acc_mean = [&](int i, int k) -> double& {
    if constexpr (ACfg::kReg) return rmean[kW * i + k];
    else if constexpr (ACfg::kLds) return lds_acc[(kW * i + k) * 256 + threadIdx.x];
    else return a.mean[(int64_t)L::dim(sub, i, k) * N + c];
  };
  auto acc_m2 = [&](int i, int k) -> double& {
    if constexpr (ACfg::kReg) return rm2[kW * i + k];
    else if constexpr (ACfg::kLds) return lds_acc[(L::NL + kW * i + k) * 256 + threadIdx.x];
    else return a.m2[(int64_t)L::dim(sub, i, k) * N + c];
  };
  if (accum) {
    if constexpr (ACfg::kReg || ACfg::kLds) {
#pragma unroll
      for (int i = 0; i < L::NCL; ++i)
#pragma unroll
        for (int k = 0; k < kW; ++k) {
          int64_t o = (int64_t)L::dim(sub, i, k) * N + c;
          acc_mean(i, k) = L::valid(sub, i, k) ? a.mean[o] : 0.0;
          acc_m2(i, k) = L::valid(sub, i, k) ? a.m2[o] : 0.0;
        }
    }
#pragma unroll
    for (int l = 0; l < NH; ++l) {
      hcm(l) = a.hm_m[(int64_t)(sub + P * l) * N + c];
      hcs(l) = a.hm_s[(int64_t)(sub + P * l) * N + c];
    }
  }
  // fold the parked record of the group starting at record R0 (R0 % P == 0)
  auto hm_flush = [&](int64_t R0) __attribute__((always_inline)) {
    const int li = (int)((R0 & 7) / P);
    if (hm_pok) {
      if constexpr (kHmLds) {
        hm_update(hcm(li), hcs(li), hm_pv);             // li is wave-uniform (record index)
      } else {
#pragma unroll
        for (int l = 0; l < NH; ++l)
          if (l == li) hm_update(hcm(l), hcs(l), hm_pv);
      }
    }
    hm_pok = false;
  };

  int64_t next_rec = a.next_rec, r = a.next_r;
  // the Welford weight of the next record is loaded one record ahead: loaded where it is used,
  // its L2 latency sat exposed in every step (the table holds one entry past rec_end)
  double inv_pf = 0.0;
  if (accum) inv_pf = welford_weight(a, r - a.next_r0);
  auto record = [&](int64_t R) __attribute__((always_inline)) {
    int64_t s = R - a.rec_base;
    if ((a.flags & RUNF_RECORD_X) && active) {
      // opaque row pitch: left visible, the compiler hoists the per-dim record addresses out of
      // the step loop (two registers per dim) for this rarely taken path
      int64_t n = N;
      asm volatile("" : "+s"(n));
      double* px = a.rec_x + s * D * n + c;
#pragma unroll
      for (int i = 0; i < L::NCL; ++i)
#pragma unroll
        for (int k = 0; k < kW; ++k)
          if (L::valid(sub, i, k)) px[L::dim(sub, i, k) * n] = x[kW * i + k];
    }
    if ((a.flags & RUNF_RECORD_LLP) && active && sub == 0) {
      a.rec_ll[s * N + c] = ll;
      a.rec_lp[s * N + c] = lp;
    }
    if (accum) {
      const double inv = inv_pf;                      // 1/(R+1), host IEEE division
      inv_pf = welford_weight(a, R + 1 - a.next_r0);
#pragma unroll
      for (int i = 0; i < L::NCL; ++i)
#pragma unroll
        for (int k = 0; k < kW; ++k) {
          if (!L::valid(sub, i, k)) continue;
          if constexpr (!ACfg::kLds && !ACfg::kReg) { if (!active) continue; }
          double& mu = acc_mean(i, k);
          double& m2 = acc_m2(i, k);
          const double xv = x[kW * i + k];
          const double delta = xv - mu;
          const double mnew = fma(delta, inv, mu);
          m2 = fma(delta, xv - mnew, m2);
          mu = mnew;
        }
      const int jr = (int)(R & (P - 1));
      if (sub == jr) {
        hm_pv = -ll;
        hm_pok = true;
      }
      if (jr == P - 1) hm_flush(R - (P - 1));
    }
  };

  if (a.flags & RUNF_RECORD_INITIAL) {
    record(r);
    ++r;
  }

  double lu_own = 0.0;
  // UNI (isotropic proposal scale, one box for every dim): the scale and the box are kernel
  // arguments (SGPRs), so the lane's likelihood constants fit in registers for the whole launch.
  // kKdReg (kD proposal on P > 1 lanes, DIAG / SHELL / FLAT): the lane's likelihood constants,
  // normaliser and prior box are registers too -- a handful per lane; staged in LDS they were a
  // read and an lgkmcnt wait on every step's likelihood
  constexpr bool kKdReg = PROP == MCG_PROP_KD_INTERP && P > 1;
  static_assert(!kKdReg || LIK == MCG_LIK_FLAT || LIK == MCG_LIK_DIAG_GAUSS || LIK == MCG_LIK_GAUSS_SHELL,
                "kD on P > 1 lanes: FLAT, DIAG_GAUSS or GAUSS_SHELL");
  constexpr bool kUniReg = UNI == 1 || UNI == 2;
  constexpr int kRc = (kUniReg || kKdReg) ? L::NL : 1;
  double rc_m[kRc], rc_i[kRc];
  // UNI: the likelihood normaliser and the box's log density in VGPRs too (a per-step cached
  // load of each put a vector-memory wait on every step's critical path)
  double rc_c = 0.0, rc_lp = 0.0;
  if constexpr (kUniReg || kKdReg) {
    rc_c = LIK == MCG_LIK_DIAG_GAUSS ? a.lik[2 * D] : LIK == MCG_LIK_GAUSS_SHELL ? a.lik[D + 2] : 0.0;
    rc_lp = a.prior_kind != MCG_PRIOR_FLAT && a.prior_kind != MCG_PRIOR_DIAG_GAUSS ? a.pri[2 * D] : 0.0;
    asm volatile("" : "+v"(rc_c), "+v"(rc_lp));
#pragma unroll
    for (int i = 0; i < L::NCL; ++i)
#pragma unroll
      for (int k = 0; k < kW; ++k) {
        const int d = L::valid(sub, i, k) ? L::dim(sub, i, k) : 0;
        rc_m[kW * i + k] = LIK == MCG_LIK_FLAT ? 0.0 : a.lik[d];
        rc_i[kW * i + k] = LIK == MCG_LIK_DIAG_GAUSS ? a.lik[D + d] : 0.0;
      }
  }
  // kKdReg: the shell's radius and inverse width, and the prior box per lane dim
  double rc_r = 0.0, rc_iw = 0.0;
  double rc_lo[kKdReg ? L::NL : 1], rc_hi[kKdReg ? L::NL : 1];
  if constexpr (kKdReg) {
    if constexpr (LIK == MCG_LIK_GAUSS_SHELL) {
      rc_r = a.lik[D];
      rc_iw = a.lik[D + 1];
    }
    const bool pbox = a.prior_kind == MCG_PRIOR_BOX || a.prior_kind == MCG_PRIOR_OPEN_BOX;
#pragma unroll
    for (int i = 0; i < L::NCL; ++i)
#pragma unroll
      for (int k = 0; k < kW; ++k) {
        const int d = L::valid(sub, i, k) ? L::dim(sub, i, k) : 0;
        rc_lo[kW * i + k] = pbox ? (a.ubox ? a.box_lo : a.pri[d]) : 0.0;
        rc_hi[kW * i + k] = pbox ? (a.ubox ? a.box_hi : a.pri[D + d]) : 0.0;
      }
  }
  // kD independence proposal: a step's draw depends on the RNG only (the picked training point's
  // leaf, its box, a uniform point in it), so they are loaded ahead: KDA = 1, the leaf of step
  // t + 2 and the box and log q of step t + 1 while step t computes; KDA = 2 (the step loop
  // unrolled by two, one register slot per step parity), the leaf of step t + 4 and the box of
  // step t + 2; P > 1 with at most 4 dims a lane (registers to spare) KDA = 4 (kKdAhead), the
  // leaf of step t + 8 and the box of step t + 4 -- the loads of 8 steps in flight per lane,
  // where 4 left 38 % of C4's wave-cycles waiting on them (round 5 PMC).  The same values as
  // loading them in the step.  (kKdAhead = 8, in groups of 4, measured 6 % slower at C4.)
  // (P > 1: lane `sub` holds the box bounds of its own dims, local slot j at kd_lo[j], kd_hi[j])
  constexpr int KDN = PROP == MCG_PROP_KD_INTERP ? L::NL : 1;
  constexpr int KDA = PROP == MCG_PROP_KD_INTERP ? (P > 1 && L::NL * kKdAhead <= 16 ? kKdAhead : P > 1 && L::NL <= 4 ? 4 : 2) : 1;
  // kd_group's steps per group: half the slots where there are 8 (a group's boxes were issued a
  // whole group earlier), else all of them
  constexpr int KDG = KDA >= 8 ? KDA / 2 : KDA;
  int kd_leaf_n[KDA];
  double kd_lo[KDA][KDN], kd_hi[KDA][KDN];
  double kd_lqp[KDA];
  auto kd_pick = [&](uint64_t Tp) __attribute__((always_inline)) -> uint32_t {
    const u32x4 w = rng(gid, (uint32_t)Tp, CALL_KD_PICK, TAG_MH, (uint32_t)(Tp >> 32));
    return randint(w.x, w.y, (uint32_t)a.kd_M);
  };
  auto kd_pick_leaf = [&](uint64_t Tp) __attribute__((always_inline)) -> int { return a.kd_pt_leaf[kd_pick(Tp)]; };
  // P > 1: the picks are staggered over the chain's lanes like the accept uniforms: at the first
  // step t of each group of P steps, lane `sub` draws the pick of step t + 2 KDA + sub, and step
  // t + q (which prefetches the leaf of step t + q + 2 KDA) takes it from lane q -- one pick per
  // P lane-steps instead of one per lane-step
  uint32_t pick_own = 0;
  auto bcast_u32 = [&](uint32_t v, int q) __attribute__((always_inline)) -> uint32_t {
    if constexpr (P == 4) {
      return q == 0 ? quad_bcast_u32<0>(v) : q == 1 ? quad_bcast_u32<1>(v) : q == 2 ? quad_bcast_u32<2>(v)
                                                                                  : quad_bcast_u32<3>(v);
    } else {
      return (uint32_t)__shfl((int)v, (lane & ~(P - 1)) | q, 64);
    }
  };
  auto kd_load_box = [&](int leaf, auto slot_c) __attribute__((always_inline)) {
    constexpr int sl = decltype(slot_c)::value;
    const double* __restrict__ bx = a.kd_box + (int64_t)leaf * 2 * D;
#pragma unroll
    for (int i = 0; i < (PROP == MCG_PROP_KD_INTERP ? L::NCL : 0); ++i)
#pragma unroll
      for (int k = 0; k < kW; ++k) {
        const int d = L::valid(sub, i, k) ? L::dim(sub, i, k) : 0;
        kd_lo[sl][kW * i + k] = bx[d];
        kd_hi[sl][kW * i + k] = bx[D + d];
      }
    kd_lqp[sl] = a.kd_logq[leaf];
  };
  // the uniforms of a step's box draw (dims 2c and 2c + 1 from call c; the lane's own blocks),
  // drawn one step ahead
  double kd_u[KDN];
  auto kd_uniforms = [&](uint64_t Tu) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < (PROP == MCG_PROP_KD_INTERP ? L::NCL : 0); ++i)
#pragma unroll
      for (int h = 0; h < kW / 2; ++h) {
        const int j = kW * i + 2 * h;
        if (!L::valid(sub, i, 2 * h)) continue;
        const u32x4 v = rng(gid, (uint32_t)Tu, (uint32_t)(L::dim(sub, i, 2 * h) >> 1), TAG_MH, (uint32_t)(Tu >> 32));
        kd_u[j] = u53(v.x, v.y);
        if (L::valid(sub, i, 2 * h + 1)) kd_u[j + 1] = u53(v.z, v.w);
      }
  };
  if constexpr (PROP == MCG_PROP_KD_INTERP) {
    // every prologue load (state, constants, accumulators) completes here, before the prefetches
    // go out: a constant whose load was still pending at the step loop's entry made the wait
    // counts inside the loop lose track of the prefetches, and the first step of every unrolled
    // group waited for all of them (vmcnt(0))
    __builtin_amdgcn_s_waitcnt(0);
    if (a.nsteps > 0) {
      // issued in the loop's own order (per slot: box, log q, the leaf KDA steps later), so the
      // wait counts at the loop entry agree with those of the loop's back edge
      int leaf0[KDA];
#pragma unroll
      for (int s = 0; s < KDA; ++s) leaf0[s] = kd_pick_leaf(a.step_base + s);
      static_for<KDA>([&](auto s_c) __attribute__((always_inline)) {
        constexpr int sl = decltype(s_c)::value;
        kd_load_box(leaf0[sl], s_c);
        kd_leaf_n[sl] = kd_pick_leaf(a.step_base + KDA + sl);
      });
    }
  }
  // log u of step t (mcmc.ml:49).  P > 1: staggered accept uniforms -- at the first step of each
  // group of P steps, lane `sub` of the chain draws log u for step t + sub; step t + q reads it
  // from lane q (one DPP broadcast, or a shuffle at P = 8)
  auto accept_lu = [&](const int q, uint64_t T) __attribute__((always_inline)) -> double {
    if constexpr (P == 1) {
      const u32x4 wa = rng(gid, (uint32_t)T, CALL_ACCEPT, TAG_MH, (uint32_t)(T >> 32));
      return plog(u53(wa.x, wa.y), s_lt);
    } else {
      if (q == 0) {
        const uint64_t Tj = T + (uint64_t)sub;
        const u32x4 wa = rng(gid, (uint32_t)Tj, CALL_ACCEPT, TAG_MH, (uint32_t)(Tj >> 32));
        lu_own = plog(u53(wa.x, wa.y), s_lt);
      }
      if constexpr (P == 4) {
        return q == 0 ? quad_bcast_f64<0>(lu_own) : q == 1 ? quad_bcast_f64<1>(lu_own)
             : q == 2 ? quad_bcast_f64<2>(lu_own) : quad_bcast_f64<3>(lu_own);
      } else if constexpr (P == 2) {
        return q == 0 ? pair_bcast_f64<0>(lu_own) : pair_bcast_f64<1>(lu_own);
      } else {
        return __shfl(lu_own, (lane & ~(P - 1)) | q, 64);
      }
    }
  };
  // kKdReg: eval_lik / eval_prior of the lane's dims on the register constants (the same
  // operations as eval_lik / eval_prior)
  auto kd_reg_lik = [&](const double* yv) __attribute__((always_inline)) -> double {
    if constexpr (!kKdReg || LIK == MCG_LIK_FLAT) {
      return 0.0;
    } else {
      double S;
      if constexpr (kW == 2) {
        double e[2];
#pragma unroll
        for (int k = 0; k < 2; ++k)
          e[k] = LIK == MCG_LIK_DIAG_GAUSS ? fma(yv[k], rc_i[k], -rc_m[k]) : yv[k] - rc_m[k];
        S = reduce_canon_w2<P>(e[0], e[1], sub);
      } else {
        double A[L::NA];
#pragma unroll
        for (int j = 0; j < L::NA; ++j) A[j] = 0.0;
#pragma unroll
        for (int i = 0; i < L::NCL; ++i)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (!L::valid(sub, i, k)) continue;
            const double e = LIK == MCG_LIK_DIAG_GAUSS ? fma(yv[4 * i + k], rc_i[4 * i + k], -rc_m[4 * i + k])
                                                       : yv[4 * i + k] - rc_m[4 * i + k];
            A[i % L::NA] = fma(e, e, A[i % L::NA]);
          }
        S = reduce_canon<P>(A);
      }
      if constexpr (LIK == MCG_LIK_DIAG_GAUSS) {
        return rc_c - 0.5 * S;
      } else {
        const double rr = psqrt(S);
        const double qq = (rr - rc_r) * rc_iw;
        return rc_c - 0.5 * qq * qq;
      }
    }
  };
  auto kd_reg_gauss_prior = [&](const double* yv) __attribute__((always_inline)) -> double {
    typedef const __attribute__((address_space(4))) double kconst;
    kconst* kpri = (kconst*)a.pri;
    asm volatile("" : "+s"(kpri));
    return eval_gauss_prior<D, P, kconst*, kW>(yv, sub, a, kpri);
  };
  auto kd_reg_box_prior = [&](const double* yv) __attribute__((always_inline)) -> double {
    int inb = 1;
#pragma unroll
    for (int i = 0; i < L::NCL; ++i)
#pragma unroll
      for (int k = 0; k < kW; ++k) {
        if (!L::valid(sub, i, k)) continue;
        const double v = yv[kW * i + k];
        if constexpr (kKdReg) inb &= (int)(v >= rc_lo[kW * i + k]) & (int)(v <= rc_hi[kW * i + k]);
      }
    inb = and_lanes<P>(inb);
    return inb ? rc_lp : -__builtin_inf();
  };
  auto kd_reg_prior = [&](const double* yv) __attribute__((always_inline)) -> double {
    if (a.prior_kind == MCG_PRIOR_FLAT) return 0.0;
    if (a.prior_kind == MCG_PRIOR_DIAG_GAUSS) return kd_reg_gauss_prior(yv);
    return kd_reg_box_prior(yv);
  };
  // the accept of step t (mcmc.ml:42-56) from its proposal's terms, then the kD prefetch into
  // the step's slot, the bitmap row and the record
  auto mh_accept = [&](int64_t t, uint64_t T, const int tq, auto par_c, const double* yv, double lly, double lpy,
                       double lqy, double lf, double lb, double lu, auto rec_c,
                       auto pick_c) __attribute__((always_inline)) {
    constexpr int par = decltype(par_c)::value;
    const double post_y = lly + lpy;
    const double post_x = ll + lp;
    const double ratio = ((post_y - post_x) + lb) - lf;
    const bool acc = lu < ratio;
    if (acc) {
#pragma unroll
      for (int j = 0; j < L::NL; ++j) x[j] = yv[j];
      ll = lly;
      lp = lpy;
      lq = lqy;
      ++na;
    }
    if constexpr (PROP == MCG_PROP_KD_INTERP) {
      // the box and log q of step t + KDA into this step's slot (its leaf arrived KDA steps
      // ago), and the leaf of step t + 2 KDA.  Issued after the accept, where the slot's old
      // log q (this step's lqy) is dead: issued before it, old and new log q were live together,
      // and the register allocator rotated the slots with copies at the loop latch that waited
      // for the fresh loads, i.e. for every prefetch in flight
      kd_load_box(kd_leaf_n[par], std::integral_constant<int, par>{});
      if constexpr (P == 1) {
        kd_leaf_n[par] = kd_pick_leaf(T + 2 * KDA);
      } else {
        // (pick_c: the caller drew this group's picks ahead, kd_group)
        if constexpr (!decltype(pick_c)::value) {
          if (tq == 0) pick_own = kd_pick(T + 2 * KDA + (uint64_t)sub);
        }
        kd_leaf_n[par] = a.kd_pt_leaf[bcast_u32(pick_own, tq)];
      }
    }
    if (a.flags & RUNF_RECORD_ACCEPT) {
      const uint64_t m = compress_ballot<P>((uint64_t)__ballot(acc && active));
      const int64_t wave = tid >> 6;
      if (lane == 0 && wave * (64 / P) < N) {
        uint8_t* row = a.bits + (a.t0 + t) * a.bits_row_bytes;
        const int64_t byte = wave * (8 / P);
        if constexpr (P == 1) *(uint64_t*)(row + byte) = m;
        else if constexpr (P == 2) *(uint32_t*)(row + byte) = (uint32_t)m;
        else if constexpr (P == 4) *(uint16_t*)(row + byte) = (uint16_t)m;
        else row[byte] = (uint8_t)m;
      }
    }
    if constexpr (decltype(rec_c)::value) {
      const int64_t tt1 = a.t0 + t + 1;
      if (tt1 == next_rec && r < a.rec_end) {
        record(r);
        ++r;
        next_rec += a.nskip;
      }
    }
  };
  // one MH step (mcmc.ml:37-56); par: the step's parity, a compile-time slot of the kD prefetch
  auto mh_step = [&](int64_t t, auto par_c, auto q_c) __attribute__((always_inline)) {
    constexpr int par = decltype(par_c)::value;
    constexpr int kq = decltype(q_c)::value;           // t mod P when the caller knows it, else -1
    const uint64_t T = a.step_base + (uint64_t)t;
    // t mod P, the step's place in its group of P (staggered draws); a compile-time constant
    // where the unrolled slots cover whole groups
    const int tq = kq >= 0 ? kq : (KDA > 1 && KDA % P == 0) ? par % P : (int)(t & (P - 1));
    const uint32_t tlo = (uint32_t)T, thi = (uint32_t)(T >> 32);
    double lf = 0.0, lb = 0.0, lqy = 0.0;
    // Re-read the (tiny, cache-resident) model constants every step: opaque pointers stop the
    // compiler from hoisting D*5 doubles into registers, which would cap occupancy.
    // They are global-memory pointers (address space 1) through the asm: an opaque generic
    // pointer would make every constant a flat load, which also counts against the LDS counter.
    typedef const __attribute__((address_space(1))) double gconst;
    gconst* glik = (gconst*)a.lik;
    gconst* gpri = (gconst*)a.pri;
    gconst* gprop = (gconst*)a.prop;
    // (the fused step with UNI constants reads none of them: no per-step copies there)
    if constexpr (!(kSeparable && kUniReg)) asm volatile("" : "+s"(glik), "+s"(gpri), "+s"(gprop));
    [[maybe_unused]] const double* qlik = (const double*)glik;
    [[maybe_unused]] const double* qpri = (const double*)gpri;
    const double* qprop = (const double*)gprop;
    double lly, lpy;
    if constexpr (kSeparable) {
      // fused: per Philox call -> 4 normals -> 4 proposed coordinates -> their terms of the
      // canonical sum and of the box test.  Keeps only x, y and 8/P accumulators live.
      typedef const __attribute__((address_space(1))) double gdouble;
      gdouble* qlik = (gdouble*)a.lik;
      gdouble* qpri = (gdouble*)a.pri;
      gdouble* qprop = (gdouble*)a.prop;
      if constexpr (!UNI) asm volatile("" : "+s"(qlik), "+s"(qpri), "+s"(qprop));
      double A[L::NA];
#pragma unroll
      for (int j = 0; j < L::NA; ++j) A[j] = 0.0;
      // box test as a lane predicate (SGPR masks), one VGPR bit for the cross-lane AND
      bool ok = true;
      const bool box = a.prior_kind != MCG_PRIOR_FLAT;
      // the lane's Philox calls of this step (c2 = call index sub + P i) advanced together
      u32x4 wl[L::NCL];
      {
        uint32_t cidx[L::NCL];
#pragma unroll
        for (int i = 0; i < L::NCL; ++i) cidx[i] = (uint32_t)(sub + P * i);
        philox_multi<L::NCL, true>(wl, gid, tlo, cidx, (TAG_MH << 16) | (thi & 0xFFFFu), rng.k0, rng.k1);
      }
      // the coordinates and terms of call i from its four normals
      auto dims1 = [&](const int i, const int k, const double zk) __attribute__((always_inline)) {
        const int cc = sub + P * i;
        if (!L::valid(sub, i, k)) return;
        const int d = 4 * cc + k;
        const double yv = fma(UNI ? a.uni_s : qprop[d], zk, x[kW * i + k]);
        y[kW * i + k] = yv;
        double rcm = 0.0, rci = 0.0;
        if constexpr (UNI) {
          rcm = rc_m[kW * i + k];
          rci = rc_i[kW * i + k];
        }
        if constexpr (LIK == MCG_LIK_DIAG_GAUSS) {
          const double e = UNI ? fma(yv, rci, -rcm) : fma(yv, qlik[D + d], -qlik[d]);
          A[i % L::NA] = fma(e, e, A[i % L::NA]);
        } else if constexpr (LIK == MCG_LIK_GAUSS_SHELL) {
          const double e = yv - (UNI ? rcm : qlik[d]);
          A[i % L::NA] = fma(e, e, A[i % L::NA]);
        }
        if constexpr (UNI == 2) {
          ok = ok & (__builtin_fabs(yv) <= a.uni_hi);
        } else {
          const double lo = UNI ? a.uni_lo : qpri[d], hi = UNI ? a.uni_hi : qpri[D + d];
          ok = ok & (yv >= lo) & (yv <= hi);
        }
      };
      auto dims = [&](const int i, const double* z) __attribute__((always_inline)) {
        const int cc = sub + P * i;
#pragma unroll
        for (int k = 0; k < kW; ++k) {
          if (!L::valid(sub, i, k)) continue;
          const int d = 4 * cc + k;
          const double yv = fma(UNI ? a.uni_s : qprop[d], z[k], x[kW * i + k]);
          y[kW * i + k] = yv;
          double rcm = 0.0, rci = 0.0;
          if constexpr (UNI) {
            rcm = rc_m[kW * i + k];
            rci = rc_i[kW * i + k];
          }
          if constexpr (LIK == MCG_LIK_DIAG_GAUSS) {
            const double e = UNI ? fma(yv, rci, -rcm)
                                 : fma(yv, qlik[D + d], -qlik[d]);   // (y - mu)/sigma
            A[i % L::NA] = fma(e, e, A[i % L::NA]);
          } else if constexpr (LIK == MCG_LIK_GAUSS_SHELL) {
            const double e = yv - (UNI ? rcm : qlik[d]);
            A[i % L::NA] = fma(e, e, A[i % L::NA]);
          }
          // branch-free closed-box test: the host stores an OPEN box as its closed equivalent
          // [nextafter(lo, +inf), nextafter(hi, -inf)] and pads FLAT priors with (-inf, inf)
          if constexpr (UNI == 2) {
            ok = ok & (__builtin_fabs(yv) <= a.uni_hi);
          } else {
            const double lo = UNI ? a.uni_lo : qpri[d], hi = UNI ? a.uni_hi : qpri[D + d];
            ok = ok & (yv >= lo) & (yv <= hi);
          }
        }
      };
      if constexpr (Shape::kPipe) {
        // one normal at a time with its table rows gathered one normal ahead: the gathers of
        // normal m + 1 are in flight while normal m is finished and its dim's terms computed
        auto word = [&](int m) __attribute__((always_inline)) -> uint32_t {
          const u32x4 w = wl[m >> 2];
          const int k = m & 3;
          return k == 0 ? w.x : k == 1 ? w.y : k == 2 ? w.z : w.w;
        };
        constexpr int NM = 4 * L::NCL;
        NrmPending q[2];
        q[0] = pnormal_issue(word(0), s_nt);
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          if (m + 1 < NM) q[(m + 1) & 1] = pnormal_issue(word(m + 1), s_nt);
          dims1(m >> 2, m & 3, pnormal_finish(q[m & 1]));
        }
      } else
#pragma unroll
      for (int i = 0; i < L::NCL; ++i) {
        double z[4];
        if constexpr (Shape::kBatchNormals) {
          pnormal4_lds(wl[i], s_nt, z);
        } else {
          const u32x4 w = wl[i];
          z[0] = pnormal(w.x, s_nt);
          z[1] = pnormal(w.y, s_nt);
          z[2] = pnormal(w.z, s_nt);
          z[3] = pnormal(w.w, s_nt);
        }
        dims(i, z);
      }
      if constexpr (LIK == MCG_LIK_FLAT) {
        lly = 0.0;
      } else {
        const double S = reduce_canon<P>(A);
        if constexpr (LIK == MCG_LIK_DIAG_GAUSS) {
          lly = (UNI ? rc_c : qlik[2 * D]) - 0.5 * S;
        } else {
          const double rr = psqrt(S);
          const double qq = (rr - qlik[D]) * qlik[D + 1];
          lly = (UNI ? rc_c : qlik[D + 2]) - 0.5 * qq * qq;
        }
      }
      const int inb = and_lanes<P>(ok ? 1 : 0);
      lpy = !box ? 0.0 : (inb ? (UNI ? rc_lp : qpri[2 * D]) : -__builtin_inf());
    } else {
      // ---- proposal (jump_proposal, mcmc.ml:41) ----
      if constexpr (PROP == MCG_PROP_GAUSS) {
#pragma unroll
        for (int i = 0; i < L::NCL; ++i) {
          const int cc = sub + P * i;
          if (P == 1 && 4 * i >= D) continue;
          const u32x4 w = rng(gid, tlo, (uint32_t)cc, TAG_MH, thi);
          double z[4];
          z[0] = pnormal(w.x, s_nt);
          z[1] = pnormal(w.y, s_nt);
          z[2] = pnormal(w.z, s_nt);
          z[3] = pnormal(w.w, s_nt);
#pragma unroll
          for (int k = 0; k < kW; ++k)
            if (L::valid(sub, i, k)) y[kW * i + k] = fma(qprop[L::dim(sub, i, k)], z[k], x[kW * i + k]);
        }
      } else if constexpr (PROP == MCG_PROP_WRAP_UNIFORM) {
        // dims 2c and 2c + 1 from Philox call c, the lane's own four-dim blocks (one lane: every
        // dim; P lanes: blocks sub, sub + P, ... -- the same draws, so any split is bit-identical)
        static_assert(kW == 4, "WRAP: four-dim lane blocks");
#pragma unroll
        for (int i = 0; i < L::NCL; ++i)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            if (!L::valid(sub, i, 2 * h)) continue;
            const int d = L::dim(sub, i, 2 * h), j = 4 * i + 2 * h;
            const u32x4 w = rng(gid, tlo, (uint32_t)(d >> 1), TAG_MH, thi);
            y[j] = wrap_uniform(qprop[d], qprop[D + d], qprop[2 * D + d], x[j], u53(w.x, w.y));
            if (L::valid(sub, i, 2 * h + 1))
              y[j + 1] = wrap_uniform(qprop[d + 1], qprop[D + d + 1], qprop[2 * D + d + 1], x[j + 1],
                                      u53(w.z, w.w));
          }
      } else if constexpr (PROP == MCG_PROP_KD_INTERP) {
        static_assert(P == 1 || D % (kW * P) == 0, "KD: P lanes need D % WP == 0");
        // Interpolate_pdf.draw (interpolate_pdf.ml:114-119) from the leaf and box loaded ahead;
        // dims 2c and 2c + 1 from call c (lane `sub`: the calls of its 4-dim blocks)
        kd_uniforms(T);
        const double* klo = kd_lo[par];
        const double* khi = kd_hi[par];
        bool strict = true;
#pragma unroll
        for (int j = 0; j < L::NL; ++j) {
          if (!L::valid(sub, j >> 2, j & 3)) continue;
          y[j] = klo[j] + (khi[j] - klo[j]) * kd_u[j];
          strict = strict && (y[j] > klo[j]) && (y[j] < khi[j]);
        }
        if constexpr (P > 1) strict = and_lanes<P>(strict ? 1 : 0) != 0;
        // strictly inside its leaf box: that leaf (see below), whose log q came with the box
        lqy = kd_lqp[par];
        if (!strict) {
          if constexpr (P == 1) {
            lqy = a.kd_logq[kd_find_leaf<D>(a.kd_nodes, a.kd_root, y)];
          } else {
            // (rare: a draw rounded onto a face) the descent needs every dim of the proposal
            double yf[D];
#pragma unroll
            for (int o = 0; o < P; ++o)
#pragma unroll
              for (int i = 0; i < L::NCL; ++i)
#pragma unroll
                for (int k = 0; k < kW; ++k)
                  if (L::valid(o, i, k)) yf[L::dim(o, i, k)] = __shfl(y[kW * i + k], (lane & ~(P - 1)) | o, 64);
            lqy = a.kd_logq[kd_find_leaf<D>(a.kd_nodes, a.kd_root, yf)];
          }
          // consumed here, so the load completes inside this rare branch (left pending at the
          // join, the wait counts after it lost track of the prefetches in flight)
          asm volatile("" : "+v"(lqy));
        }
        // (the box and log q of step t + KDA go out after this step's accept: kd_prefetch)
        lf = lqy;   // log_jump_prob start proposed = log q(proposed)
        lb = lq;    // log_jump_prob proposed start = log q(start)
      }
      else if constexpr (PROP == MCG_PROP_DE) {
        static_assert(kW == 4, "DE: four-dim lane blocks");
        // Mcmc.differential_evolution_proposal (mcmc.ml:198-218) over the caller's samples:
        // pick_samples i != j (:199-203; j drawn from the n - 1 others, no retry loop), the scale
        // 1.0 with probability mode_hopping_frac (no draw consulted when it is 0, :209) else
        // N(0, 2.38 / sqrt(2 D)) (:212-213), z' = z + d (y_j - x_i) (:214-217).  The samples are
        // rows of D doubles (two row gathers per step, L2-resident); log_jump_prob = 0.
        const uint32_t nde = (uint32_t)a.de_M;
        const u32x4 wi = rng(gid, tlo, CALL_DE_IDX, TAG_MH, thi);
        const uint32_t ii = randint(wi.x, wi.y, nde);
        const uint32_t jj = randint(wi.z, wi.w, nde - 1u);
        const uint32_t jd = jj + (jj >= ii ? 1u : 0u);
        const u32x4 ws = rng(gid, tlo, CALL_DE_SCALE, TAG_MH, thi);
        const double mh = qprop[0];
        const double dsc = (mh != 0.0 && u53(ws.x, ws.y) < mh) ? 1.0 : qprop[1] * pnormal(ws.z, s_nt);
        const double* __restrict__ si = a.de_pts + (int64_t)ii * D;
        const double* __restrict__ sj = a.de_pts + (int64_t)jd * D;
        // every lane draws the same indices and scale; lane `sub` moves its own dims
#pragma unroll
        for (int i = 0; i < L::NCL; ++i)
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (L::valid(sub, i, k)) {
              const int d = L::dim(sub, i, k);
              y[4 * i + k] = x[4 * i + k] + dsc * (sj[d] - si[d]);
            }
      }
      else if constexpr (PROP == MCG_PROP_MIXTURE) {
        static_assert(P == 1, "MIXTURE: one lane per chain");
        // pick a component: Random.float 1.0 walked down the normalised weights (mcmc.ml:168-173);
        // (a u past the last weight cannot occur: mcg_set_proposal refuses weights whose walk
        // lets the largest draw fall through, pack_mixture)
        using M = MixLayout<D>;
        const int nc = (int)qprop[0];
        const u32x4 ws = rng(gid, tlo, CALL_MIX, TAG_MH, thi);
        double u = u53(ws.x, ws.y);
        int pick = nc - 1;
        for (int cc = 0; cc < nc; ++cc) {
          const double p = M::comp(qprop, cc)[0];
          if (u < p) { pick = cc; break; }
          u = u - p;
        }
        const double* m = M::comp(qprop, pick);
        const int kind = (int)m[2];
        int leaf_y = -1;
        if (kind == MCG_MIX_GAUSS) {
#pragma unroll
          for (int i = 0; i < L::NCL; ++i) {
            if (4 * i >= D) continue;
            const u32x4 w = rng(gid, tlo, (uint32_t)i, TAG_MH, thi);
            double z[4];
            z[0] = pnormal(w.x, s_nt);
            z[1] = pnormal(w.y, s_nt);
            z[2] = pnormal(w.z, s_nt);
            z[3] = pnormal(w.w, s_nt);
#pragma unroll
            for (int k = 0; k < kW; ++k)
              if (kW * i + k < D) y[kW * i + k] = fma(m[5 + kW * i + k], z[k], x[kW * i + k]);
          }
        } else if (kind == MCG_MIX_KD_INTERP) {
          const u32x4 w = rng(gid, tlo, CALL_KD_PICK, TAG_MH, thi);
          const int leaf = a.kd_pt_leaf[randint(w.x, w.y, (uint32_t)a.kd_M)];
          const double* __restrict__ bx = a.kd_box + (int64_t)leaf * 2 * D;
          bool strict = true;
#pragma unroll
          for (int d = 0; d < D; d += 2) {
            const u32x4 v = rng(gid, tlo, (uint32_t)(d >> 1), TAG_MH, thi);
            y[d] = bx[d] + (bx[D + d] - bx[d]) * u53(v.x, v.y);
            strict = strict && (y[d] > bx[d]) && (y[d] < bx[D + d]);
            if (d + 1 < D) {
              y[d + 1] = bx[d + 1] + (bx[D + d + 1] - bx[d + 1]) * u53(v.z, v.w);
              strict = strict && (y[d + 1] > bx[d + 1]) && (y[d + 1] < bx[D + d + 1]);
            }
          }
          if (strict) leaf_y = leaf;
        } else {
          // SHIFT_UNIFORM: x + random_between a b; WRAP_UNIFORM: Mcmc.uniform_wrapping
#pragma unroll
          for (int d = 0; d < D; d += 2) {
            const u32x4 w = rng(gid, tlo, (uint32_t)(d >> 1), TAG_MH, thi);
            const double u0 = u53(w.x, w.y), u1 = u53(w.z, w.w);
            if (kind == MCG_MIX_SHIFT_UNIFORM) {
              y[d] = x[d] + (m[5 + d] + m[5 + 2 * D + d] * u0);
              if (d + 1 < D) y[d + 1] = x[d + 1] + (m[5 + d + 1] + m[5 + 2 * D + d + 1] * u1);
            } else {
              y[d] = wrap_uniform(m[5 + d], m[5 + D + d], m[5 + 2 * D + d], x[d], u0);
              if (d + 1 < D) y[d + 1] = wrap_uniform(m[5 + d + 1], m[5 + D + d + 1], m[5 + 2 * D + d + 1], x[d + 1], u1);
            }
          }
        }
        if (mix_kd) lqy = a.kd_logq[leaf_y >= 0 ? leaf_y : kd_find_leaf<D>(a.kd_nodes, a.kd_root, y)];
        lf = mix_log_jp<D>(qprop, x, y, lqy, s_lt);   // log_jump_prob start proposed
        lb = mix_log_jp<D>(qprop, y, x, lq, s_lt);    // log_jump_prob proposed start
      }
      if constexpr (kKdReg) {
        // eval_lik / eval_prior of the lane's dims on the register constants (the same operations)
        lly = kd_reg_lik(y);
        lpy = kd_reg_prior(y);
      } else {
        // likelihood / prior constants through scalar loads (the scalar cache and lgkmcnt, not
        // a per-step vmcnt wait behind the proposal's loads)
        typedef const __attribute__((address_space(4))) double kconst;
        kconst* klik = (kconst*)a.lik;
        kconst* kpri = (kconst*)a.pri;
        asm volatile("" : "+s"(klik), "+s"(kpri));
        lly = eval_lik<D, P, LIK, kconst*, kW>(y, sub, a, klik);
        lpy = eval_prior<D, P, kconst*, kW>(y, sub, a, kpri);
      }
    }
    // ---- Hastings ratio and accept test (mcmc.ml:42-56) ----
    const double lu = accept_lu(tq, T);
    mh_accept(t, T, tq, par_c, y, lly, lpy, lqy, lf, lb, lu, std::true_type{}, std::false_type{});
  };
  // kD proposal on P > 1 lanes, KDA steps at a time (round 6).  The independence proposal's draw,
  // its log q and the proposal's likelihood and prior do not depend on the chain state, so the
  // KDA steps' proposals are evaluated together (branch-free across the steps, the rare face
  // descents and the prior kind hoisted out: one basic block the scheduler interleaves), then
  // the KDA accepts run in order.  The same operations as mh_step, step for step.
  constexpr bool kKdGroup = kKdReg && KDA >= 4 && KDG % P == 0;
  // group of KDG steps t0 .. t0 + KDG - 1 on prefetch slots B .. B + KDG - 1
  auto kd_group = [&](int64_t t0, auto b_c) __attribute__((always_inline)) {
    constexpr int B = decltype(b_c)::value;
    constexpr int G = KDG;
    double yg[G][L::NL];
    double lqg[G], llg[G], lpg[G], lug[G];
    int stg[G];
    static_for<G>([&](auto s_c) __attribute__((always_inline)) {
      constexpr int sl = decltype(s_c)::value;
      kd_uniforms(a.step_base + (uint64_t)(t0 + sl));
      bool strict = true;
#pragma unroll
      for (int j = 0; j < L::NL; ++j) {
        yg[sl][j] = 0.0;
        if (!L::valid(sub, j >> 2, j & 3)) continue;
        yg[sl][j] = kd_lo[B + sl][j] + (kd_hi[B + sl][j] - kd_lo[B + sl][j]) * kd_u[j];
        strict = strict && (yg[sl][j] > kd_lo[B + sl][j]) && (yg[sl][j] < kd_hi[B + sl][j]);
      }
      stg[sl] = and_lanes<P>(strict ? 1 : 0);
      lqg[sl] = kd_lqp[B + sl];
    });
    // the picks of steps t0 + 2 KDA .. (staggered: lane sub draws step t0 + 2 KDA + q P + sub for
    // the q-th group of P steps), drawn here beside the other draws instead of inside the accepts
    uint32_t pickg[G / P > 0 ? G / P : 1];
#pragma unroll
    for (int q = 0; q < G / P; ++q) pickg[q] = kd_pick(a.step_base + (uint64_t)(t0 + 2 * KDA + q * P + sub));
    static_for<G>([&](auto s_c) __attribute__((always_inline)) {
      constexpr int sl = decltype(s_c)::value;
      if (!stg[sl]) {
        double yf[D];
#pragma unroll
        for (int o = 0; o < P; ++o)
#pragma unroll
          for (int i = 0; i < L::NCL; ++i)
#pragma unroll
            for (int k = 0; k < kW; ++k)
              if (L::valid(o, i, k)) yf[L::dim(o, i, k)] = __shfl(yg[sl][kW * i + k], (lane & ~(P - 1)) | o, 64);
        double v = a.kd_logq[kd_find_leaf<D>(a.kd_nodes, a.kd_root, yf)];
        asm volatile("" : "+v"(v));                     // completes inside the rare branch
        lqg[sl] = v;
      }
    });
#pragma unroll
    for (int sl = 0; sl < G; ++sl) llg[sl] = kd_reg_lik(yg[sl]);
    if (a.prior_kind == MCG_PRIOR_FLAT) {
#pragma unroll
      for (int sl = 0; sl < G; ++sl) lpg[sl] = 0.0;
    } else if (a.prior_kind == MCG_PRIOR_DIAG_GAUSS) {
#pragma unroll
      for (int sl = 0; sl < G; ++sl) lpg[sl] = kd_reg_gauss_prior(yg[sl]);
    } else {
#pragma unroll
      for (int sl = 0; sl < G; ++sl) lpg[sl] = kd_reg_box_prior(yg[sl]);
    }
#pragma unroll
    for (int sl = 0; sl < G; ++sl) lug[sl] = accept_lu(sl % P, a.step_base + (uint64_t)(t0 + sl));
    // every step of the group records, and only into the moments and harmonic-mean partials (the
    // C4 shape): the G accepts run back to back, then the G records from the states they left --
    // the same updates in the same order as record() after each step, without a branch between
    // the accepts
    const bool rec_all = accum && (a.flags & (RUNF_RECORD_X | RUNF_RECORD_LLP)) == 0 && a.nskip == 1 &&
                         next_rec == a.t0 + t0 + 1 && r + G <= a.rec_end;
    if (rec_all) {
      double xs[G][L::NL], lls[G];
      static_for<G>([&](auto s_c) __attribute__((always_inline)) {
        constexpr int sl = decltype(s_c)::value;
        // log_jump_prob start proposed = log q(proposed); proposed start = log q(start), the
        // state after step t0 + sl - 1
        if constexpr (sl % P == 0) pick_own = pickg[sl / P];
        mh_accept(t0 + sl, a.step_base + (uint64_t)(t0 + sl), sl % P, std::integral_constant<int, B + sl>{},
                  yg[sl], llg[sl], lpg[sl], lqg[sl], lqg[sl], lq, lug[sl], std::false_type{}, std::true_type{});
#pragma unroll
        for (int j = 0; j < L::NL; ++j) xs[sl][j] = x[j];
        lls[sl] = ll;
      });
#pragma unroll
      for (int sl = 0; sl < G; ++sl) {
        const double inv = inv_pf;                     // 1/(R+1), host IEEE division
        inv_pf = welford_weight(a, r + sl + 1 - a.next_r0);
#pragma unroll
        for (int i = 0; i < L::NCL; ++i)
#pragma unroll
          for (int k = 0; k < kW; ++k) {
            if (!L::valid(sub, i, k)) continue;
            if constexpr (!ACfg::kLds && !ACfg::kReg) { if (!active) continue; }
            double& mu = acc_mean(i, k);
            double& m2 = acc_m2(i, k);
            const double xv = xs[sl][kW * i + k];
            const double delta = xv - mu;
            const double mnew = fma(delta, inv, mu);
            m2 = fma(delta, xv - mnew, m2);
            mu = mnew;
          }
      }
#pragma unroll
      for (int sl = 0; sl < G; ++sl) {
        const int64_t R = r + sl;
        const int jr = (int)(R & (P - 1));
        if (sub == jr) {
          hm_pv = -lls[sl];
          hm_pok = true;
        }
        if (jr == P - 1) hm_flush(R - (P - 1));
      }
      r += G;
      next_rec += G;
    } else {
      static_for<G>([&](auto s_c) __attribute__((always_inline)) {
        constexpr int sl = decltype(s_c)::value;
        if constexpr (sl % P == 0) pick_own = pickg[sl / P];
        mh_accept(t0 + sl, a.step_base + (uint64_t)(t0 + sl), sl % P, std::integral_constant<int, B + sl>{},
                  yg[sl], llg[sl], lpg[sl], lqg[sl], lqg[sl], lq, lug[sl], std::true_type{}, std::true_type{});
      });
    }
  };
  if constexpr (KDA > 1) {
    // step t uses prefetch slot t mod KDA: the loop unrolled by KDA, then the last nsteps mod KDA
    // steps on slots 0, 1, ...
    int64_t t = 0;
    if constexpr (kKdGroup) {
      for (; t + KDA - 1 < a.nsteps; t += KDA)
        static_for<KDA / KDG>([&](auto g_c) __attribute__((always_inline)) {
          kd_group(t + decltype(g_c)::value * KDG, std::integral_constant<int, decltype(g_c)::value * KDG>{});
        });
    } else {
      for (; t + KDA - 1 < a.nsteps; t += KDA)
        static_for<KDA>([&](auto s_c) __attribute__((always_inline)) {
          mh_step(t + decltype(s_c)::value, s_c, std::integral_constant<int, -1>{});
        });
    }
    const int64_t t_end = t;
    static_for<KDA - 1>([&](auto s_c) __attribute__((always_inline)) {
      if (t_end + decltype(s_c)::value < a.nsteps)
        mh_step(t_end + decltype(s_c)::value, s_c, std::integral_constant<int, -1>{});
    });
  } else if constexpr (kStepUnroll && P > 1) {
    // the loop unrolled by P: each step's place in its group of P (staggered accept uniforms) is
    // a compile-time constant
    int64_t t = 0;
    for (; t + P - 1 < a.nsteps; t += P)
      static_for<P>([&](auto s_c) __attribute__((always_inline)) {
        mh_step(t + decltype(s_c)::value, std::integral_constant<int, 0>{}, s_c);
      });
    for (; t < a.nsteps; ++t) mh_step(t, std::integral_constant<int, 0>{}, std::integral_constant<int, -1>{});
  } else {
    for (int64_t t = 0; t < a.nsteps; ++t)
      mh_step(t, std::integral_constant<int, 0>{}, std::integral_constant<int, -1>{});
  }

  if (!active) return;
  // opaque row pitch: the prologue's per-dim addresses would otherwise be kept live through the
  // step loop for these stores (two registers per address)
  int64_t n = N;
  asm volatile("" : "+s"(n));
#pragma unroll
  for (int i = 0; i < L::NCL; ++i)
#pragma unroll
    for (int k = 0; k < kW; ++k)
      if (L::valid(sub, i, k)) a.x[(int64_t)L::dim(sub, i, k) * n + c] = x[kW * i + k];
  if (sub == 0) {
    a.ll[c] = ll;
    a.lp[c] = lp;
    a.nacc[c] += na;
  }
  if (accum) {
    if constexpr (ACfg::kReg || ACfg::kLds) {
#pragma unroll
      for (int i = 0; i < L::NCL; ++i)
#pragma unroll
        for (int k = 0; k < kW; ++k)
          if (L::valid(sub, i, k)) {
            int64_t o = (int64_t)L::dim(sub, i, k) * n + c;
            a.mean[o] = acc_mean(i, k);
            a.m2[o] = acc_m2(i, k);
          }
    }
    // a partial group at the end of the launch: fold it now (the classes keep record order)
    hm_flush((r - 1) & ~(int64_t)(P - 1));
#pragma unroll
    for (int l = 0; l < NH; ++l) {
      a.hm_m[(int64_t)(sub + P * l) * n + c] = hcm(l);
      a.hm_s[(int64_t)(sub + P * l) * n + c] = hcs(l);
    }
  }
}

// evaluate ll, lp of the initial states (mcmc.ml:59-61)
template <int D, int LIK>
__global__ void __launch_bounds__(256) eval_kernel(const MhArgs a) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.N) return;
  double x[Layout<D, 1>::NL];
#pragma unroll
  for (int d = 0; d < Layout<D, 1>::NL; ++d) x[d] = d < D ? a.x[(int64_t)d * a.N + c] : 0.0;
  a.ll[c] = eval_lik<D, 1, LIK>(x, 0, a, a.lik);
  a.lp[c] = eval_prior<D, 1>(x, 0, a, a.pri);
}

template <int D, int LIK>
hipError_t launch_eval(const MhArgs& a, hipStream_t s) {
  const int64_t grid = (a.N + 255) / 256;
  hipLaunchKernelGGL((eval_kernel<D, LIK>), dim3((unsigned)grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int D, int P, int LIK, int PROP>
hipError_t launch_mh(const MhArgs& a, int64_t nthreads, hipStream_t s) {
  const int block = MhShape<D, P, LIK, PROP>::kBlock;
  const int64_t grid = (nthreads + block - 1) / block;
  constexpr int lds = AccumCfg<D, P, lane_width<D, P, PROP>()>::kLdsBytes;
  if constexpr (separable<LIK, PROP>()) {
    if (a.prior_kind == MCG_PRIOR_DIAG_GAUSS) {
      hipLaunchKernelGGL((mh_kernel<D, P, LIK, PROP, kUniGaussPrior>), dim3((unsigned)grid), dim3(block), lds, s, a);
      return hipGetLastError();
    }
    if (a.uni && a.uni_lo == -a.uni_hi) {
      hipLaunchKernelGGL((mh_kernel<D, P, LIK, PROP, 2>), dim3((unsigned)grid), dim3(block), lds, s, a);
      return hipGetLastError();
    }
    if (a.uni) {
      hipLaunchKernelGGL((mh_kernel<D, P, LIK, PROP, 1>), dim3((unsigned)grid), dim3(block), lds, s, a);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((mh_kernel<D, P, LIK, PROP, 0>), dim3((unsigned)grid), dim3(block), lds, s, a);
  return hipGetLastError();
}

}  // namespace mcg
