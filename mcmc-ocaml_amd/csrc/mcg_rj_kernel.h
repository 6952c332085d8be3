// mcg_rj_kernel.h -- batched reversible-jump MH between two models (Mcmc.make_rjmcmc_sampler,
// mcmc.ml:89-119, driven by rjmcmc_array's schedule mcmc.ml:121-139).
//
// One lane per chain.  The chain carries a model tag (0 = A, 1 = B) and a point padded with zeros
// to DM = max(D_A, D_B); every model block on the device is padded to DM the same way
// (mcg_rj.cpp), so a model of dimension D_m < DM evaluates exactly as at D_m: the padded terms
// add +0 to the canonical sums and the padded box bounds are (-inf, inf).
//
// Device descriptor (double[]): per model m a 16-double header at 16 m
//   [0] D_m  [1] log p_m  [2] p_m  [3] lik kind  [4] prior kind  [5] jump kind  [6] into kind
//   [7] lik block offset  [8] prior block offset  [9] jump block offset  [10] into block offset
// blocks: likelihood in the MH kernel's layout at DM; prior [lo, hi, lp_in, lo, hi] at DM (a
// DIAG_GAUSS prior: [mu/s, 1/s, C, mu, s] at DM, zero-padded);
// jumps: GAUSS s[DM]; WRAP lo, hi, dx [DM]; INDEP_GAUSS mu[DM], s[DM], 1/s[DM], mu/s[DM], C.
#pragma once
#include "mcg_mh_kernel.h"

namespace mcg {

constexpr uint32_t CALL_RJ = 0xFFFF0006u, CALL_RJ_START = 0xFFFF0007u;

template <int DM>
__device__ __forceinline__ double rj_lik(const double* y, const MhArgs& a, int kind, const double* q) {
  switch (kind) {
    case MCG_LIK_DIAG_GAUSS: return eval_lik<DM, 1, MCG_LIK_DIAG_GAUSS>(y, 0, a, q);
    case MCG_LIK_GAUSS_SHELL: return eval_lik<DM, 1, MCG_LIK_GAUSS_SHELL>(y, 0, a, q);
    case MCG_LIK_FULLCOV_GAUSS: return eval_lik<DM, 1, MCG_LIK_FULLCOV_GAUSS>(y, 0, a, q);
    default: return 0.0;
  }
}

// lpa / lpb (mcmc.ml:116-118): FLAT, a box, or Stats.log_multi_gaussian mu sigma (DIAG_GAUSS:
// the DIAG_GAUSS likelihood's canonical constants padded to DM with zeros, so the pad dims add +0)
template <int DM>
__device__ __forceinline__ double rj_prior(const double* y, const MhArgs& a, int kind, const double* q) {
  if (kind == MCG_PRIOR_FLAT) return 0.0;
  if (kind == MCG_PRIOR_DIAG_GAUSS) return eval_lik<DM, 1, MCG_LIK_DIAG_GAUSS>(y, 0, a, q);
  int inb = 1;
#pragma unroll
  for (int d = 0; d < DM; ++d) inb &= (int)(y[d] >= q[d]) & (int)(y[d] <= q[DM + d]);
  return inb ? q[2 * DM] : -__builtin_inf();
}

// log_jump_prob _ to of an independence jump (INDEP_GAUSS / KD); 0 for the random walks
template <int DM>
__device__ __forceinline__ double rj_ljp_to(const double* to, int Dm, int kind, const double* q,
                                            const KdView& kd, int leaf_hint) {
  if (kind == MCG_RJ_JUMP_INDEP_GAUSS) {
    // sum_d Stats.log_gaussian mu_d s_d to_d (stats.ml:98-101) = C - 1/2 sum_d e_d^2
    double S = 0.0;
#pragma unroll
    for (int d = 0; d < DM; ++d)
      if (d < Dm) {
        const double e = fma(to[d], q[2 * DM + d], -q[3 * DM + d]);
        S = fma(e, e, S);
      }
    return q[4 * DM] - 0.5 * S;
  } else if (kind == MCG_RJ_JUMP_KD) {
    const int leaf = leaf_hint >= 0 ? leaf_hint : kd_find_leaf<DM>(kd.nodes, kd.root, to);
    return kd.logq[leaf];
  }
  return 0.0;
}

// draw a jump of `kind` from x into y (dims < Dm); returns the kD leaf of y when known (a draw
// strictly inside its leaf box), else -1
template <int DM>
__device__ __forceinline__ int rj_draw(const double* x, double* y, int Dm, int kind, const double* q,
                                       const KdView& kd, const Rng& rng, uint32_t gid, uint32_t tlo,
                                       uint32_t thi, const double2* lt, const double2* nt) {
#pragma unroll
  for (int d = 0; d < DM; ++d) y[d] = 0.0;
  if (kind == MCG_RJ_JUMP_GAUSS || kind == MCG_RJ_JUMP_INDEP_GAUSS) {
#pragma unroll
    for (int i = 0; 4 * i < DM; ++i) {
      const u32x4 w = rng(gid, tlo, (uint32_t)i, TAG_MH, thi);
      double z[4];
      z[0] = pnormal(w.x, nt);
      z[1] = pnormal(w.y, nt);
      z[2] = pnormal(w.z, nt);
      z[3] = pnormal(w.w, nt);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int d = 4 * i + k;
        if (d < DM && d < Dm) {
          if (kind == MCG_RJ_JUMP_GAUSS) y[d] = fma(q[d], z[k], x[d]);        // x + s z
          else y[d] = fma(q[DM + d], z[k], q[d]);                              // mu + s z
        }
      }
    }
    return -1;
  } else if (kind == MCG_RJ_JUMP_WRAP) {
#pragma unroll
    for (int d = 0; d < DM; d += 2) {
      if (d >= Dm) continue;
      const u32x4 w = rng(gid, tlo, (uint32_t)(d >> 1), TAG_MH, thi);
      y[d] = wrap_uniform(q[d], q[DM + d], q[2 * DM + d], x[d], u53(w.x, w.y));
      if (d + 1 < DM && d + 1 < Dm)
        y[d + 1] = wrap_uniform(q[d + 1], q[DM + d + 1], q[2 * DM + d + 1], x[d + 1], u53(w.z, w.w));
    }
    return -1;
  } else {
    // Interpolate_pdf.draw (interpolate_pdf.ml:114-119); boxes of a D_m-dim tree, stride 2 D_m
    const u32x4 w = rng(gid, tlo, CALL_KD_PICK, TAG_MH, thi);
    const int leaf = kd.pt_leaf[randint(w.x, w.y, (uint32_t)kd.M)];
    const double* __restrict__ bx = kd.box + (int64_t)leaf * 2 * Dm;
    bool strict = true;
#pragma unroll
    for (int d = 0; d < DM; d += 2) {
      if (d >= Dm) continue;
      const u32x4 v = rng(gid, tlo, (uint32_t)(d >> 1), TAG_MH, thi);
      y[d] = bx[d] + (bx[Dm + d] - bx[d]) * u53(v.x, v.y);
      strict = strict && (y[d] > bx[d]) && (y[d] < bx[Dm + d]);
      if (d + 1 < DM && d + 1 < Dm) {
        y[d + 1] = bx[d + 1] + (bx[Dm + d + 1] - bx[d + 1]) * u53(v.z, v.w);
        strict = strict && (y[d + 1] > bx[d + 1]) && (y[d + 1] < bx[Dm + d + 1]);
      }
    }
    return strict ? leaf : -1;
  }
}

template <int DM>
__global__ void __launch_bounds__(256) rj_kernel(const MhArgs a) {
  __shared__ double2 s_lt[kLogTabN];
  __shared__ double2 s_nt[kNrmTabN];
  for (int i = threadIdx.x; i < kLogTabN; i += blockDim.x) s_lt[i] = kLogTab[i];
  for (int i = threadIdx.x; i < kNrmTabN; i += blockDim.x) s_nt[i] = kNrmTab[i];
  __syncthreads();
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = tid < a.N;
  const int64_t c = active ? tid : 0;
  const int64_t N = a.N;
  const Rng rng{a.k0, a.k1};
  const uint32_t gid = a.chain_offset + (uint32_t)c;
  const int lane = threadIdx.x & 63;
  const double* __restrict__ H = a.rj;

  double x[DM], y[DM];
#pragma unroll
  for (int d = 0; d < DM; ++d) x[d] = a.x[(int64_t)d * N + c];
  double ll = a.ll[c], lp = a.lp[c];
  int tag = a.tag[c];
  unsigned long long na = 0, nb_rec = 0;

  int64_t next_rec = a.next_rec, r = a.next_r;
  auto record = [&](int64_t R) {
    const int64_t s = R - a.rec_base;
    if ((a.flags & RUNF_RECORD_X) && active) {
#pragma unroll
      for (int d = 0; d < DM; ++d) a.rec_x[(s * DM + d) * N + c] = x[d];
    }
    if ((a.flags & RUNF_RECORD_LLP) && active) {
      a.rec_ll[s * N + c] = ll;
      a.rec_lp[s * N + c] = lp;
      a.rec_tag[s * N + c] = (uint8_t)tag;
    }
    nb_rec += (unsigned long long)tag;
  };
  if (a.flags & RUNF_RECORD_INITIAL) {
    record(r);
    ++r;
  }

  for (int64_t t = 0; t < a.nsteps; ++t) {
    const uint64_t T = a.step_base + (uint64_t)t;
    const uint32_t tlo = (uint32_t)T, thi = (uint32_t)(T >> 32);
    // ---- jump_proposal (mcmc.ml:92-102): internal with prob p_tag, else into the other model ----
    const u32x4 ws = rng(gid, tlo, CALL_RJ, TAG_MH, thi);
    const double* hm = H + 16 * tag;
    const bool internal = u53(ws.x, ws.y) < hm[2];
    const int ytag = internal ? tag : 1 - tag;
    const double* hy = H + 16 * ytag;
    const int Dy = (int)hy[0];
    const int jk = internal ? (int)hy[5] : (int)hy[6];
    const double* jq = H + (int64_t)(internal ? hy[9] : hy[10]);
    const int leaf = rj_draw<DM>(x, y, Dy, jk, jq, a.rj_kd[ytag], rng, gid, tlo, thi, s_lt, s_nt);
    // ---- log_jump_prob (mcmc.ml:103-112) ----
    double lf, lb;
    if (internal) {
      lf = hy[1] + rj_ljp_to<DM>(y, Dy, jk, jq, a.rj_kd[ytag], leaf);
      lb = hy[1] + rj_ljp_to<DM>(x, Dy, jk, jq, a.rj_kd[ytag], -1);
    } else {
      const int bk = (int)hm[6];
      const double* bq = H + (int64_t)hm[10];
      lf = hy[1] + rj_ljp_to<DM>(y, Dy, jk, jq, a.rj_kd[ytag], leaf);
      lb = hm[1] + rj_ljp_to<DM>(x, (int)hm[0], bk, bq, a.rj_kd[tag], -1);
    }
    // ---- log_like / log_prior of the proposed model (mcmc.ml:113-118) ----
    const double lly = rj_lik<DM>(y, a, (int)hy[3], H + (int64_t)hy[7]);
    const double lpy = hy[1] + rj_prior<DM>(y, a, (int)hy[4], H + (int64_t)hy[8]);
    const double ratio = (((lly + lpy) - (ll + lp)) + lb) - lf;
    const u32x4 wa = rng(gid, tlo, CALL_ACCEPT, TAG_MH, thi);
    const bool acc = plog(u53(wa.x, wa.y), s_lt) < ratio;
    if (acc) {
#pragma unroll
      for (int d = 0; d < DM; ++d) x[d] = y[d];
      ll = lly;
      lp = lpy;
      tag = ytag;
      ++na;
    }
    if (a.flags & RUNF_RECORD_ACCEPT) {
      const uint64_t m = (uint64_t)__ballot(acc && active);
      const int64_t wave = tid >> 6;
      if (lane == 0 && wave * 64 < N) *(uint64_t*)(a.bits + (a.t0 + t) * a.bits_row_bytes + wave * 8) = m;
    }
    const int64_t tt1 = a.t0 + t + 1;
    if (tt1 == next_rec && r < a.rec_end) {
      record(r);
      ++r;
      next_rec += a.nskip;
    }
  }
  if (!active) return;
#pragma unroll
  for (int d = 0; d < DM; ++d) a.x[(int64_t)d * N + c] = x[d];
  a.ll[c] = ll;
  a.lp[c] = lp;
  a.tag[c] = (uint8_t)tag;
  a.nacc[c] += na;
  if (a.flags & RUNF_ACCUMULATE) a.rj_nb[c] += nb_rec;
}

// rjmcmc_array's start (mcmc.ml:123-128): the fair coin per chain when no tags are given, the
// start point of the chain's model (xa [D_A][N] or xb [D_B][N]), then ll, lp (with log p_model)
template <int DM>
__global__ void __launch_bounds__(256) rj_init_kernel(const MhArgs a, int draw_tags, const double* xa,
                                                      const double* xb) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.N) return;
  const uint32_t gid = a.chain_offset + (uint32_t)c;
  int tag = a.tag[c];
  if (draw_tags) {
    const Rng rng{a.k0, a.k1};
    const u32x4 w = rng(gid, (uint32_t)a.step_base, CALL_RJ_START, TAG_MH, (uint32_t)(a.step_base >> 32));
    tag = u53(w.x, w.y) < 0.5 ? 0 : 1;
    a.tag[c] = (uint8_t)tag;
  }
  const double* h = a.rj + 16 * tag;
  const int Dm = (int)h[0];
  const double* src = tag ? xb : xa;
  double x[DM];
#pragma unroll
  for (int d = 0; d < DM; ++d) {
    x[d] = d < Dm ? src[(int64_t)d * a.N + c] : 0.0;
    a.x[(int64_t)d * a.N + c] = x[d];
  }
  a.ll[c] = rj_lik<DM>(x, a, (int)h[3], a.rj + (int64_t)h[7]);
  a.lp[c] = rj_prior<DM>(x, a, (int)h[4], a.rj + (int64_t)h[8]) + h[1];
}

template <int DM>
hipError_t launch_rj(const MhArgs& a, int64_t nthreads, hipStream_t s) {
  hipLaunchKernelGGL((rj_kernel<DM>), dim3((unsigned)((nthreads + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int DM>
hipError_t launch_rj_init(const MhArgs& a, int draw_tags, const double* xa, const double* xb, hipStream_t s) {
  hipLaunchKernelGGL((rj_init_kernel<DM>), dim3((unsigned)((a.N + 255) / 256)), dim3(256), 0, s, a, draw_tags,
                     xa, xb);
  return hipGetLastError();
}

}  // namespace mcg
