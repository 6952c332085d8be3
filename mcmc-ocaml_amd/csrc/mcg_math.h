// mcg_math.h -- device RNG and portable fp64 math for gfx950.
//
// The operation sequence of every function here is the RNG/math spec of DESIGN.md §RNG; the
// CPU oracle (oracle/oracle.c) restates the same spec independently, so a kernel and the
// oracle produce bit-identical variates.  Compile with -ffp-contract=off: every fused
// multiply-add below is an explicit fma().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mcg_tables.h"

namespace mcg {

// ---- Philox4x32-10 (Salmon, Moraes, Dror, Shaw 2011) ----
struct u32x4 { uint32_t x, y, z, w; };

// a ^ b ^ c in one VALU op: gfx950 v_bitop3_b32 with truth table 0x96 (hipcc emits two v_xor_b32)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}

__device__ __forceinline__ u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                        uint32_t k0, uint32_t k1) {
  // keep the 20 round keys out of long-lived SGPRs: recompute them (SALU adds) per call
  asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;   // v_mad_u64_u32
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0);
    uint32_t n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  return u32x4{c0, c1, c2, c3};
}

// N Philox4x32-10 calls that differ only in the third counter word (the MH step's per-dim
// calls: same chain, step and tag), advanced round by round together: N independent chains of
// (v_mad_u64_u32 -> v_bitop3) instead of one serial 10-round chain after another, so one wave
// keeps its SIMD issuing; the shared first-round product of c0 is computed once.
// kUniform: c1 and c3 are the same in every lane (the MH step's step counter and tag); their
// first-round xor with the key then runs on the scalar unit, and each lane does one v_xor with
// an SGPR operand (v_bitop3 takes one scalar operand, so xor3(v, s, s) costs a v_mov as well)
template <int N, bool kUniform = false>
__device__ __forceinline__ void philox_multi(u32x4* out, uint32_t c0, uint32_t c1, const uint32_t* c2,
                                             uint32_t c3, uint32_t k0, uint32_t k1) {
  asm volatile("" : "+s"(k0), "+s"(k1));
  uint32_t a[N], b[N], c[N], d[N];
  {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint32_t c1k = 0, c3k = 0;
    if constexpr (kUniform) {
      c1k = (uint32_t)__builtin_amdgcn_readfirstlane((int)(c1 ^ k0));
      c3k = (uint32_t)__builtin_amdgcn_readfirstlane((int)(c3 ^ k1));
    }
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2[n];
      a[n] = kUniform ? ((uint32_t)(p1 >> 32) ^ c1k) : xor3((uint32_t)(p1 >> 32), c1, k0);
      b[n] = (uint32_t)p1;
      c[n] = kUniform ? ((uint32_t)(p0 >> 32) ^ c3k) : xor3((uint32_t)(p0 >> 32), c3, k1);
      d[n] = (uint32_t)p0;
    }
  }
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * a[n];
      const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[n];
      const uint32_t n0 = xor3((uint32_t)(p1 >> 32), b[n], k0);
      const uint32_t n2 = xor3((uint32_t)(p0 >> 32), d[n], k1);
      b[n] = (uint32_t)p1;
      d[n] = (uint32_t)p0;
      a[n] = n0;
      c[n] = n2;
    }
  }
#pragma unroll
  for (int n = 0; n < N; ++n) out[n] = u32x4{a[n], b[n], c[n], d[n]};
}

// counter layout (c0, c1, c2, (tag << 16) | hi16), key = seed
enum : uint32_t {
  TAG_MH = 1u, TAG_NEST_WALK = 3u, TAG_NEST_PRIOR = 4u, TAG_POSTERIOR = 5u,
  CALL_ACCEPT = 0xFFFF0000u, CALL_DE_IDX = 0xFFFF0001u, CALL_DE_SCALE = 0xFFFF0002u,
  CALL_KD_PICK = 0xFFFF0003u, CALL_START = 0xFFFF0004u, CALL_MIX = 0xFFFF0005u
};

struct Rng {
  uint32_t k0, k1;
  __device__ __forceinline__ u32x4 operator()(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t tag,
                                               uint32_t hi16) const {
    return philox(c0, c1, c2, (tag << 16) | (hi16 & 0xFFFFu), k0, k1);
  }
};

__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }
__device__ __forceinline__ double bitsd(uint64_t b) { return __longlong_as_double((long long)b); }

// (2m+1) 2^-53 for the 52-bit m = w0:w1[31:12].  Built exactly from the bits:
// (1 + m 2^-52) - (1 - 2^-53) is exact (Sterbenz), so this equals the spec's int->double form.
__device__ __forceinline__ double u53(uint32_t w0, uint32_t w1) {
  const uint32_t hi = 0x3FF00000u | (w0 >> 12);
  const uint32_t lo = (w0 << 20) | (w1 >> 12);
  return bitsd(((uint64_t)hi << 32) | lo) - (1.0 - 0x1p-53);
}

// (a + 1/2) 2^-32 exactly: (1 + a 2^-32) - (1 - 2^-33)
__device__ __forceinline__ double u32_open(uint32_t a) {
  const uint32_t hi = 0x3FF00000u | (a >> 12);
  const uint32_t lo = a << 20;
  return bitsd(((uint64_t)hi << 32) | lo) - (1.0 - 0x1p-33);
}

__device__ __forceinline__ uint32_t randint(uint32_t w0, uint32_t w1, uint32_t n) {
  uint64_t u = ((uint64_t)w0 << 32) | (uint64_t)w1;
  return (uint32_t)__umul64hi(u, (uint64_t)n);
}

// A 64-bit constant materialised in an SGPR pair at its point of use (two s_mov): left to the
// compiler, a kernel whose loop calls plog / pexp keeps every polynomial coefficient in a VGPR
// pair for its whole life (~30 VGPRs in the MH kernel), which costs occupancy.  Same values.
#define MCG_SCONST(c) ([&] { double v_ = (c); asm volatile("" : "+s"(v_)); return v_; }())

// log (spec v4): mantissa rounded to 8 bits, j = round(256 (m - 1)) in [0, 256];
// cells j >= kLogSplit are halved (m/2, k+1); d = m - m_j exact, r = d RN(1/m_j), |r| <= 2^-9,
// degree-6 log1p.  All reduction steps are 32-bit integer ops on the high word.
// `tab` points at kLogTab (mcg_tables.h) or at a copy staged in LDS (per-lane gather).
__device__ __forceinline__ double plog(double x, const double2* tab) {
  const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
  const uint64_t b = dbits(x);
  const uint32_t hi = (uint32_t)(b >> 32), lo = (uint32_t)b;
  const uint32_t j = ((hi & 0xFFFFFu) + 0x800u) >> 12;
  const bool big = j >= (uint32_t)kLogSplit;
  const int k = (int)(hi >> 20) - 1023 + (big ? 1 : 0);
  const uint32_t mhi = (hi & 0xFFFFFu) | (big ? 0x3FE00000u : 0x3FF00000u);
  const uint32_t chi = ((0x3FF00u + j) << 12) - (big ? 0x100000u : 0u);
  const double m = bitsd(((uint64_t)mhi << 32) | lo);
  const double mj = bitsd((uint64_t)chi << 32);
  const double2 cl = tab[j];
  const double d = m - mj;
  const double r = d * cl.x;
  const double z = r * r;
  double q = fma(r, MCG_SCONST(-0x1.5555555555555p-3), MCG_SCONST(0x1.999999999999ap-3));
  q = fma(r, q, -0.25);
  q = fma(r, q, MCG_SCONST(0x1.5555555555555p-2));
  q = fma(r, q, -0.5);
  const double p = fma(z, q, r);
  const double dk = (double)k;
  return fma(dk, MCG_SCONST(ln2_hi), cl.y) + fma(dk, MCG_SCONST(ln2_lo), p);
}

__device__ __forceinline__ double plog(double x) { return plog(x, kLogTab); }

// exp for x <= 0; 0 below -708
__device__ __forceinline__ double pexp(double x) {
  const double inv_ln2 = 0x1.71547652b82fep+0;
  const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
  bool tiny = !(x > -708.0);
  x = tiny ? 0.0 : x;
  double kd = floor(fma(x, MCG_SCONST(inv_ln2), 0.5));
  double r = fma(-kd, MCG_SCONST(ln2_hi), x);
  r = fma(-kd, MCG_SCONST(ln2_lo), r);
  double p = MCG_SCONST(0x1.1eed8eff8d898p-29);
  p = fma(p, r, MCG_SCONST(0x1.ae64567f544e4p-26));
  p = fma(p, r, MCG_SCONST(0x1.27e4fb7789f5cp-22));
  p = fma(p, r, MCG_SCONST(0x1.71de3a556c734p-19));
  p = fma(p, r, MCG_SCONST(0x1.a01a01a01a01ap-16));
  p = fma(p, r, MCG_SCONST(0x1.a01a01a01a01ap-13));
  p = fma(p, r, MCG_SCONST(0x1.6c16c16c16c17p-10));
  p = fma(p, r, MCG_SCONST(0x1.1111111111111p-7));
  p = fma(p, r, MCG_SCONST(0x1.5555555555555p-5));
  p = fma(p, r, MCG_SCONST(0x1.5555555555555p-3));
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  int k = (int)kd;
  double v = p * bitsd((uint64_t)(k + 1023) << 52);
  return tiny ? 0.0 : v;
}

// sqrt (spec v3): bit-trick rsqrt seed, 4 Newton steps on 1/sqrt(a), then a * y
__device__ __forceinline__ double psqrt(double a) {
  double y = bitsd(0x5FE6EB50C7B537A9ull - (dbits(a) >> 1));
  const double ha = 0.5 * a;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double h = ha * y;
    const double e = fma(-h, y, 0.5);
    y = fma(y, e, y);
  }
  return a * y;
}

// standard normal from one 32-bit word (spec v7): the sign is bit 31; the other
// 31 bits give v = 2w + 1 (odd), u = v 2^-33 in (0, 1/2).  double(v) = 2^E (1 + f) is exact; the
// segment is (E, top kNrmS bits of f), its row bits 15..24 of the high word; the rest of f, put
// under the exponent of 1.0, is x' = 1 + t/32 exactly, and z = -+ p_seg(x'): the segment's cubic
// in x' (oracle/gen_tables.py), the same coefficients and Horner as the oracle's.  Exactly
// symmetric: flipping bit 31 negates z.  `tab` points at kNrmTab or at a copy staged in LDS:
// (e3, e2) of the segment at row r, (e1, e0) at row kNrmSeg + r -- two 16-B gathers from one
// address (constant offset), each on LDS slot r mod 16.
static_assert(kNrmS == 5 && kNrmDeg == 3, "pnormal is written for 32 segments per octave, degree 3");
constexpr int kNrmSeg = 32 << kNrmS;
static_assert(kNrmTabN == 2 * kNrmSeg, "normal table: two rows per segment");

// (w << 1) | 1 and (hi & 0x7FFF) | 0x3FF00000 as single VALU ops (hipcc emits shift + or pairs)
__device__ __forceinline__ uint32_t nrm_odd(uint32_t w) {
  uint32_t r;
  asm("v_lshl_or_b32 %0, %1, 1, 1" : "=v"(r) : "v"(w));
  return r;
}
__device__ __forceinline__ uint32_t nrm_frac_hi(uint32_t hi) {
  uint32_t r;
  // gfx9 VOP3: no literal operand and one scalar operand, so the mask comes in a VGPR
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(hi), "v"(0x7FFFu), "s"(0x3FF00000u));
  return r;
}

struct NrmPending {
  double x;
  double2 c32, c10;
  uint32_t sign;
};
__device__ __forceinline__ NrmPending pnormal_issue(uint32_t w, const double2* tab) {
  const uint32_t v = nrm_odd(w);
  const double dv = (double)v;                                   // exact
  const uint32_t hi = (uint32_t)__double2hiint(dv);
  const uint32_t lo = (uint32_t)__double2loint(dv);
  // row = bits 15..24 of hi: the low 5 bits of the biased exponent 1023 + E, then j (the table
  // is stored rotated by one octave, oracle/gen_tables.py dev_row), so no bias subtraction and
  // both gathers take the table base as an immediate offset
  const double2* c = tab + ((hi >> 15) & (uint32_t)(kNrmSeg - 1));
  NrmPending r;
  r.x = __hiloint2double((int)nrm_frac_hi(hi), (int)lo);        // x' = 1 + t/32, exact
  r.c32 = c[0];
  r.c10 = c[kNrmSeg];
  r.sign = w;
  return r;
}
__device__ __forceinline__ double pnormal_finish(const NrmPending& q) {
  double p = fma(q.c32.x, q.x, q.c32.y);
  p = fma(p, q.x, q.c10.x);
  p = fma(p, q.x, q.c10.y);
  // p_hi ^ (w & 0x80000000): the sign of the word flips z
  uint32_t h;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6c" : "=v"(h) : "v"(q.sign), "v"(__double2hiint(p)), "s"(0x80000000u));
  return __hiloint2double((int)h, __double2loint(p));
}
__device__ __forceinline__ double pnormal(uint32_t w, const double2* tab) {
  return pnormal_finish(pnormal_issue(w, tab));
}

// The four normals of one Philox call with their eight table gathers issued back to back and
// one LDS wait (the compiler, short of registers, otherwise issues two gathers, waits, and
// evaluates one normal at a time).  `tab` must be the LDS copy of kNrmTab.  The same operations
// as pnormal, so the same values.
__device__ __forceinline__ void pnormal4_lds(const u32x4 w, const double2* tab, double z[4]) {
  const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
  uint32_t ad[4];
  double xp[4];
  const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) double2*)tab;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double dv = (double)nrm_odd(ww[k]);
    const uint32_t hi = (uint32_t)__double2hiint(dv);
    ad[k] = base + ((hi >> 15) & (uint32_t)(kNrmSeg - 1)) * 16u;
    xp[k] = __hiloint2double((int)nrm_frac_hi(hi), __double2loint(dv));
  }
  double2 a0, a1, a2, a3, b0, b1, b2, b3;
  static_assert(kNrmSeg * 16 == 16384, "second half of the table at offset 16384");
  asm volatile(
      "ds_read_b128 %0, %8\n\t"
      "ds_read_b128 %4, %8 offset:16384\n\t"
      "ds_read_b128 %1, %9\n\t"
      "ds_read_b128 %5, %9 offset:16384\n\t"
      "ds_read_b128 %2, %10\n\t"
      "ds_read_b128 %6, %10 offset:16384\n\t"
      "ds_read_b128 %3, %11\n\t"
      "ds_read_b128 %7, %11 offset:16384\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3), "=&v"(b0), "=&v"(b1), "=&v"(b2), "=&v"(b3)
      : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3])
      : "memory");
  const double2 A[4] = {a0, a1, a2, a3}, B[4] = {b0, b1, b2, b3};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    NrmPending q;
    q.x = xp[k];
    q.c32 = A[k];
    q.c10 = B[k];
    q.sign = ww[k];
    z[k] = pnormal_finish(q);
  }
}

// log1p(r), r in [0,1] (Goldberg: r * log(1+r) / ((1+r)-1)); log-sum-exp on the portable
// exp/log.  Drives the running nested-sampling estimate (nested.ml:139-142).
__device__ __forceinline__ double plog1p(double r, const double2* tab = kLogTab) {
  double u = 1.0 + r;
  if (u == 1.0) return r;
  return plog(u, tab) * (r / (u - 1.0));
}

// `tab`: kLogTab or a copy staged in LDS
__device__ __forceinline__ double plse(double a, double b, const double2* tab = kLogTab) {
  if (a == -__builtin_inf() && b == -__builtin_inf()) return -__builtin_inf();
  if (b > a) {
    double t = a;
    a = b;
    b = t;
  }
  return a + plog1p(pexp(b - a), tab);
}

// log-space harmonic-mean partial (m, s) += v = -ll (evidence.ml:101-107 in log space);
// s == 0 marks an empty partial.  Branch-free form of oracle.c hm_update.
__device__ __forceinline__ void hm_update(double& m, double& s, double v) {
  const double e = (v == m) ? 1.0 : pexp(-fabs(v - m));
  const double s_up = (v > m) ? s * e + 1.0 : s + e;
  const bool empty = s == 0.0;
  s = empty ? 1.0 : s_up;
  m = (empty || v > m) ? v : m;
}

__device__ __forceinline__ void hm_comb(double& ma, double& sa, double mb, double sb) {
  if (sb == 0.0) return;
  if (sa == 0.0) { ma = mb; sa = sb; return; }
  const double mm = (ma > mb) ? ma : mb;
  sa = sa * pexp(ma - mm) + sb * pexp(mb - mm);
  ma = mm;
}

// canonical 8-accumulator reduction tree (DESIGN.md §Canonical sums)
__device__ __forceinline__ double canon8(const double* A) {
  return ((A[0] + A[4]) + (A[2] + A[6])) + ((A[1] + A[5]) + (A[3] + A[7]));
}

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
  return __shfl_xor(v, m, 64);
}

// value of lane ^ M.  M = 1, 2 stay inside a lane quad: a DPP quad_perm move (VALU, a few cycles)
// instead of ds_bpermute (an LDS round trip on the serial chain of every MH / walker step).
template <int M>
__device__ __forceinline__ int xor_lane_i(int v) {
  if constexpr (M == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);   // [1,0,3,2]
  else if constexpr (M == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
  else if constexpr (M == 4) {
    // two row shifts, each writing one half of every 8-lane group (bank_mask: banks of 4 lanes):
    // lanes 0-3 (banks 0, 2) take lane + 4 (row_shl:4), lanes 4-7 (banks 1, 3) lane - 4 (row_shr:4)
    const int t = __builtin_amdgcn_update_dpp(0, v, 0x104, 0xF, 0x5, false);
    return __builtin_amdgcn_update_dpp(t, v, 0x114, 0xF, 0xA, false);
  }
  else return __shfl_xor(v, M, 64);
}
template <int M>
__device__ __forceinline__ double xor_lane_d(double v) {
  if constexpr (M == 1 || M == 2 || M == 4) {
    return __hiloint2double(xor_lane_i<M>(__double2hiint(v)), xor_lane_i<M>(__double2loint(v)));
  } else {
    return __shfl_xor(v, M, 64);
  }
}

// broadcast lane K of each lane pair to the pair (DPP quad_perm [K, K, 2 + K, 2 + K])
template <int K>
__device__ __forceinline__ double pair_bcast_f64(double v) {
  constexpr int ctl = K | (K << 2) | ((2 + K) << 4) | ((2 + K) << 6);
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), ctl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), ctl, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// broadcast lane K of each lane quad to the quad (DPP quad_perm, no LDS)
template <int K>
__device__ __forceinline__ uint32_t quad_bcast_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xF, 0xF, false);
}
template <int K>
__device__ __forceinline__ double quad_bcast_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), K * 0x55, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), K * 0x55, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

}  // namespace mcg
