// mcg_fullcov_kernel.h -- batched MH step for the full-covariance Gaussian (BASELINE C5) with the
// quadratic form on the matrix cores.
//
// Same step as mh_kernel (mcmc.ml:37-56 driven by mcmc.ml:58-72), specialised for
// LIK = FULLCOV_GAUSS, PROP = GAUSS and D in {16, 32, 48, 64}:
//   * one wave = 16 chains x 4 lane quadrants; lane (n, q) = lane n + 16 q owns the dims
//     4 kb + q (kb = 0 .. D/4-1) of chain n -- exactly the B-operand layout of
//     v_mfma_f64_16x16x4_f64, so the proposal's residuals r = y - mu feed the matrix core with
//     no data movement;
//   * e = U r (U = upper Cholesky factor of the precision) is a (D x D) x (D x 16 chains) product:
//     row block ib (16 rows) x column block kb (4 columns) per MFMA, blocks below the diagonal
//     skipped (kb >= 4 ib), U's fragments staged in LDS in lane order (conflict-free reads);
//     the MFMA accumulates in k order with an fma per term (measured bit-exact against an fma
//     chain, scripts/probes), so e_i is the fma chain over j of the oracle (oracle.c);
//   * the MFMA output holds rows 16 ib + 4 ri + q in lane quadrant q, i.e. the same rows the lane
//     owns dims of; S = sum e_i^2 uses FULLCOV's canonical accumulator k(i) = (i & 3) |
//     ((i >> 4) & 1) << 2, which keeps every accumulator inside one lane;
//   * Philox call c still yields dims 4c .. 4c+3 (spec v4): lane q draws calls 4 m + q and a
//     4 x 4 transpose across the lane quadrants (v_permlane32_swap + v_permlane16_swap, gfx950)
//     hands every lane its dims.
#pragma once
#include "mcg_mh_kernel.h"

namespace mcg {

typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int D>
struct FcLayout {
  static_assert(D % 16 == 0 && D >= 16 && D <= 64, "MFMA full-covariance path: D in {16,32,48,64}");
  static constexpr int NKB = D / 4;      // column blocks of 4 = dims per lane
  static constexpr int NIB = D / 16;     // row blocks of 16
  static constexpr int NM = D / 16;      // Philox calls per lane (calls 4 m + q)
  static constexpr int frag(int ib, int kb) {
    int f = 0;
    for (int i = 0; i < ib; ++i) f += NKB - 4 * i;
    return f + (kb - 4 * ib);
  }
  static constexpr int NFRAG = frag(NIB, 4 * NIB);
};

// 4 x 4 transpose across the lane quadrants: on entry v[k] in quadrant q is M[q][k], on exit it
// is M[k][q].  Stage 1 swaps the upper half of v[0..1] with the lower half of v[2..3]; stage 2
// swaps the odd 16-lane rows of v[0], v[2] with the even rows of v[1], v[3].
__device__ __forceinline__ void swap32(double& a, double& b) {
  auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
  auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap16(double& a, double& b) {
  auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(a), __double2loint(b), false, false);
  auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(a), __double2hiint(b), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}
// v + v[lane ^ 32] and v + v[lane ^ 16] with the same two swaps (VALU, no ds_bpermute round
// trip on the step's serial chain): after swap32(a, b) of two copies of v, a + b holds the pair
// {v[i], v[i ^ 32]} in every lane (in either order: the sum is the same bits); likewise swap16
__device__ __forceinline__ double sum_xor32(double v) {
  double a = v, b = v;
  swap32(a, b);
  return a + b;
}
__device__ __forceinline__ double sum_xor16(double v) {
  double a = v, b = v;
  swap16(a, b);
  return a + b;
}
__device__ __forceinline__ int and_xor32_16(int v) {
  auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  v = (int)r[0] & (int)r[1];
  auto t = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return (int)t[0] & (int)t[1];
}
__device__ __forceinline__ void transpose_quadrants(double* v) {
  swap32(v[0], v[2]);
  swap32(v[1], v[3]);
  swap16(v[0], v[1]);
  swap16(v[2], v[3]);
}

// 512-thread workgroups, one per CU: eight waves = two per SIMD, sharing one copy of the tables
constexpr int kFcBlock = 512;

// Per step: the lane's four Philox calls one at a time -> 4 normals -> quadrant
// transpose -> 4 proposed coordinates; each coordinate's residual r = y - mu goes straight into
// the matrix core (row blocks ib with 4 ib <= kb, four accumulators, kb ascending per block, so
// every e_i is still the oracle's fma chain), and y itself is kept in registers until the accept
// test (a v_cndmask pair per dim).  Chain state, Welford accumulators, the proposed point and the
// four MFMA accumulators fit the 256 registers of two waves per SIMD.
// UNI: one proposal scale and one box for every dim (MhArgs::uni): scalars, no per-step loads;
// UNI == 2: the box is symmetric, [-h, h], tested as |y| <= h (mcg_mh_kernel.h)
template <int D, int UNI>
__global__ void __launch_bounds__(kFcBlock, 1) mh_fullcov_kernel(const MhArgs a) {
  using F = FcLayout<D>;
  constexpr int NL = F::NKB;
  __shared__ double2 s_lt[kLogTabN];
  __shared__ double2 s_nt[kNrmTabN];
  __shared__ double s_u[F::NFRAG * 64];
  // mu by lane quadrant, [q][kb] = mu[4 kb + q], then the likelihood normaliser C and the prior
  // box's log density (per-step global loads of these were in-order vmcnt waits on every step)
  __shared__ double s_mu[D + 2];
  for (int i = threadIdx.x; i < kLogTabN; i += blockDim.x) s_lt[i] = kLogTab[i];
  for (int i = threadIdx.x; i < kNrmTabN; i += blockDim.x) s_nt[i] = kNrmTab[i];
  for (int i = threadIdx.x; i < D; i += blockDim.x) s_mu[(i & 3) * (D / 4) + (i >> 2)] = a.lik[i];
  if (threadIdx.x == 0) {
    s_mu[D] = a.lik[D];
    s_mu[D + 1] = a.prior_kind == MCG_PRIOR_FLAT ? 0.0 : a.pri[2 * D];
  }
  {
    // U fragments in lane order: frag (ib, kb), lane l -> U[16 ib + (l & 15)][4 kb + (l >> 4)],
    // zero below the diagonal (the oracle's chains start at j = i)
    const double* __restrict__ U = a.lik + D + 1;
    for (int e = threadIdx.x; e < F::NFRAG * 64; e += blockDim.x) {
      const int f = e >> 6, l = e & 63;
      int ib = 0, rem = f;
      while (rem >= F::NKB - 4 * ib) { rem -= F::NKB - 4 * ib; ++ib; }
      const int row = 16 * ib + (l & 15), col = 4 * (4 * ib + rem) + (l >> 4);
      s_u[e] = col >= row ? U[row * D + col] : 0.0;
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4;                                // lane quadrant = sub
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t chain = wave * 16 + (lane & 15);
  const bool active = chain < a.N;
  const int64_t c = active ? chain : 0;
  const int64_t N = a.N;
  const Rng rng{a.k0, a.k1};
  const uint32_t gid = a.chain_offset + (uint32_t)c;
  auto dim = [&](int kb) { return 4 * kb + q; };

  double x[NL];
#pragma unroll
  for (int kb = 0; kb < NL; ++kb) x[kb] = a.x[(int64_t)dim(kb) * N + c];
  double ll = a.ll[c], lp = a.lp[c];
  unsigned long long na = 0;

  const bool accum = (a.flags & RUNF_ACCUMULATE) != 0;
  constexpr int P = 4, NH = 2;
  __shared__ double s_hm[2 * NH * kFcBlock];             // harmonic-mean partials [2 NH][block]
  auto hcm = [&](int l) -> double& { return s_hm[(2 * l) * kFcBlock + threadIdx.x]; };
  auto hcs = [&](int l) -> double& { return s_hm[(2 * l + 1) * kFcBlock + threadIdx.x]; };
  double hm_pv = 0.0;
  bool hm_pok = false;
  double rmean[NL], rm2[NL];
  if (accum) {
#pragma unroll
    for (int kb = 0; kb < NL; ++kb) {
      rmean[kb] = a.mean[(int64_t)dim(kb) * N + c];
      rm2[kb] = a.m2[(int64_t)dim(kb) * N + c];
    }
#pragma unroll
    for (int l = 0; l < NH; ++l) {
      hcm(l) = a.hm_m[(int64_t)(q + P * l) * N + c];
      hcs(l) = a.hm_s[(int64_t)(q + P * l) * N + c];
    }
  }
  auto hm_flush = [&](int64_t R0) {
    const int li = (int)((R0 & 7) / P);
    if (hm_pok) hm_update(hcm(li), hcs(li), hm_pv);        // li: wave-uniform
    hm_pok = false;
  };

  int64_t next_rec = a.next_rec, r = a.next_r;
  double inv_pf = 0.0;                                   // Welford weight, one record ahead
  if (accum) inv_pf = welford_weight(a, r - a.next_r0);
  auto record = [&](int64_t R) {
    const int64_t s = R - a.rec_base;
    if ((a.flags & RUNF_RECORD_X) && active) {
      // opaque row pitch: left visible, the compiler hoists the 16 per-dim record addresses out
      // of the step loop (32 registers, spilled) for this rarely taken path
      int64_t n = N;
      asm volatile("" : "+s"(n));
      double* px = a.rec_x + (s * D + q) * n + c;
#pragma unroll
      for (int kb = 0; kb < NL; ++kb) px[4 * kb * n] = x[kb];
    }
    if ((a.flags & RUNF_RECORD_LLP) && active && q == 0) {
      a.rec_ll[s * N + c] = ll;
      a.rec_lp[s * N + c] = lp;
    }
    if (accum) {
      const double inv = inv_pf;
      inv_pf = welford_weight(a, R + 1 - a.next_r0);
#pragma unroll
      for (int kb = 0; kb < NL; ++kb) {
        const double delta = x[kb] - rmean[kb];
        const double mnew = fma(delta, inv, rmean[kb]);
        rm2[kb] = fma(delta, x[kb] - mnew, rm2[kb]);
        rmean[kb] = mnew;
      }
      const int jr = (int)(R & (P - 1));
      if (q == jr) {
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
  // Philox words one call ahead: call m + 1's (or the next step's call 0) are drawn right after
  // call m's normals, so their serial rounds issue between call m's MFMAs (the matrix pipe takes
  // one per ~66 clocks from a wave) instead of ahead of the next call's normals.  The words depend
  // only on (chain, step, call), never on the chain state.
  u32x4 w_ahead = rng(gid, (uint32_t)a.step_base, (uint32_t)q, TAG_MH, (uint32_t)(a.step_base >> 32));
  for (int64_t t = 0; t < a.nsteps; ++t) {
    const uint64_t T = a.step_base + (uint64_t)t;
    const uint32_t tlo = (uint32_t)T, thi = (uint32_t)(T >> 32);
    // model constants through global (not flat) pointers: a flat load counts against the LDS
    // counter too, so every wait for one would also drain the table gathers and U fragments
    typedef const __attribute__((address_space(1))) double gdouble;
    gdouble* qpri = (gdouble*)a.pri;
    gdouble* qprop = (gdouble*)a.prop;
    asm volatile("" : "+s"(qpri), "+s"(qprop));
    // ---- proposal y = x + s z (mcmc.ml:41) fused with e = U (y - mu) on the matrix cores ----
    bool ok = true;
    double yreg[NL];
    dbl4 e[F::NIB];
#pragma unroll
    for (int ib = 0; ib < F::NIB; ++ib) e[ib] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int m = 0; m < F::NM; ++m) {
      // U fragments and mu are loop-invariant LDS reads: without a barrier the compiler hoists
      // all of them out of the step loop into ~110 registers
      asm volatile("" ::: "memory");
      double v[4];
      const u32x4 w = w_ahead;
      pnormal4_lds(w, s_nt, v);            // the four normals' eight table gathers, one LDS wait
      if (m + 1 < F::NM) {
        w_ahead = rng(gid, tlo, (uint32_t)(4 * (m + 1) + q), TAG_MH, thi);
      } else {
        const uint64_t T1 = T + 1;
        w_ahead = rng(gid, (uint32_t)T1, (uint32_t)q, TAG_MH, (uint32_t)(T1 >> 32));
      }
      transpose_quadrants(v);                 // v[k'] = z[16 m + 4 k' + q]
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) {
        const int kb = 4 * m + k2;
        const int d = dim(kb);
        const double yv = fma(UNI ? a.uni_s : qprop[d], v[k2], x[kb]);
        yreg[kb] = yv;
        if constexpr (UNI == 2) ok = ok & (__builtin_fabs(yv) <= a.uni_hi);
        else ok = ok & (yv >= (UNI ? a.uni_lo : qpri[d])) & (yv <= (UNI ? a.uni_hi : qpri[D + d]));
        const double rv = yv - s_mu[q * NL + kb];
#pragma unroll
        for (int ib = 0; ib < F::NIB; ++ib)
          if (4 * ib <= kb)
            e[ib] = __builtin_amdgcn_mfma_f64_16x16x4f64(s_u[F::frag(ib, kb) * 64 + lane], rv, e[ib], 0, 0, 0);
      }
    }
    // ---- log-likelihood: S = sum e_i^2 (accumulators k = q for even ib, k = q + 4 for odd ib) --
    double A0 = 0.0, A1 = 0.0;
#pragma unroll
    for (int ib = 0; ib < F::NIB; ++ib)
#pragma unroll
      for (int ri = 0; ri < 4; ++ri) {
        if (ib & 1) A1 = fma(e[ib][ri], e[ib][ri], A1);
        else A0 = fma(e[ib][ri], e[ib][ri], A0);
      }
    const double b = A0 + A1;
    const double cs = sum_xor32(b);
    const double S = sum_xor16(cs);
    const double lly = s_mu[D] - 0.5 * S;
    const int inb = and_xor32_16(ok ? 1 : 0);
    const double lpy = a.prior_kind == MCG_PRIOR_FLAT ? 0.0 : (inb ? s_mu[D + 1] : -__builtin_inf());
    // ---- Hastings ratio and accept test (mcmc.ml:42-56); staggered accept uniforms ----
    const double ratio = (lly + lpy) - (ll + lp);
    const int qq = (int)(t & (P - 1));
    if (qq == 0) {
      const uint64_t Tj = T + (uint64_t)q;
      const u32x4 wa = rng(gid, (uint32_t)Tj, CALL_ACCEPT, TAG_MH, (uint32_t)(Tj >> 32));
      lu_own = plog(u53(wa.x, wa.y), s_lt);
    }
    const double lu = __shfl(lu_own, (lane & 15) | (qq << 4), 64);
    const bool acc = lu < ratio;
#pragma unroll
    for (int kb = 0; kb < NL; ++kb) x[kb] = acc ? yreg[kb] : x[kb];
    if (acc) {
      ll = lly;
      lp = lpy;
      ++na;
    }
    if (a.flags & RUNF_RECORD_ACCEPT) {
      const uint64_t mb = (uint64_t)__ballot(acc && active) & 0xFFFFull;   // quadrant 0 = chains
      if (lane == 0 && wave * 16 < N) {
        uint8_t* row = a.bits + (a.t0 + t) * a.bits_row_bytes;
        *(uint16_t*)(row + wave * 2) = (uint16_t)mb;
      }
    }
    const int64_t tt1 = a.t0 + t + 1;
    if (tt1 == next_rec && r < a.rec_end) {
      record(r);
      ++r;
      next_rec += a.nskip;
    }
  }

  if (!active) return;
  // opaque row pitch: the prologue's per-dim addresses would otherwise be kept live through the
  // step loop for these stores (two registers per address, spilled)
  int64_t n = N;
  asm volatile("" : "+s"(n));
  const int64_t o = (int64_t)q * n + c;
#pragma unroll
  for (int kb = 0; kb < NL; ++kb) a.x[o + 4 * kb * n] = x[kb];
  if (q == 0) {
    a.ll[c] = ll;
    a.lp[c] = lp;
    a.nacc[c] += na;
  }
  if (accum) {
#pragma unroll
    for (int kb = 0; kb < NL; ++kb) {
      a.mean[o + 4 * kb * n] = rmean[kb];
      a.m2[o + 4 * kb * n] = rm2[kb];
    }
    hm_flush((r - 1) & ~(int64_t)(P - 1));
#pragma unroll
    for (int l = 0; l < NH; ++l) {
      a.hm_m[o + P * l * n] = hcm(l);
      a.hm_s[o + P * l * n] = hcs(l);
    }
  }
}

template <int D>
hipError_t launch_mh_fullcov(const MhArgs& a, int64_t nthreads, hipStream_t s) {
  const int64_t grid = (nthreads + kFcBlock - 1) / kFcBlock;   // nthreads = 4 N: 128 chains per block
  const dim3 g((unsigned)grid), b(kFcBlock);
  if (a.uni && a.uni_lo == -a.uni_hi) hipLaunchKernelGGL((mh_fullcov_kernel<D, 2>), g, b, 0, s, a);
  else if (a.uni) hipLaunchKernelGGL((mh_fullcov_kernel<D, 1>), g, b, 0, s, a);
  else hipLaunchKernelGGL((mh_fullcov_kernel<D, 0>), g, b, 0, s, a);
  return hipGetLastError();
}

}  // namespace mcg
