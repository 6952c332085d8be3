// mcg_math.h -- device RNG and portable fp64 math for gfx950.
//
// The operation sequence of every function here is the RNG/math spec of DESIGN.md §RNG; the
// CPU oracle (oracle/oracle.c) restates the same spec independently, so a kernel and the
// oracle produce bit-identical variates.  Compile with -ffp-contract=off: every fused
// multiply-add below is an explicit fma().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mcg {

// ---- Philox4x32-10 (Salmon, Moraes, Dror, Shaw 2011) ----
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                        uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;   // v_mad_u64_u32
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  return u32x4{c0, c1, c2, c3};
}

// counter layout (c0, c1, c2, (tag << 16) | hi16), key = seed
enum : uint32_t {
  TAG_MH = 1u, TAG_NEST_WALK = 3u, TAG_NEST_PRIOR = 4u,
  CALL_ACCEPT = 0xFFFF0000u, CALL_DE_IDX = 0xFFFF0001u, CALL_DE_SCALE = 0xFFFF0002u,
  CALL_KD_PICK = 0xFFFF0003u, CALL_START = 0xFFFF0004u
};

struct Rng {
  uint32_t k0, k1;
  __device__ __forceinline__ u32x4 operator()(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t tag,
                                               uint32_t hi16) const {
    return philox(c0, c1, c2, (tag << 16) | (hi16 & 0xFFFFu), k0, k1);
  }
};

__device__ __forceinline__ double u53(uint32_t w0, uint32_t w1) {
  uint64_t m = ((uint64_t)w0 << 20) | (uint64_t)(w1 >> 12);
  return (double)((m << 1) | 1u) * 0x1p-53;
}

__device__ __forceinline__ uint32_t randint(uint32_t w0, uint32_t w1, uint32_t n) {
  uint64_t u = ((uint64_t)w0 << 32) | (uint64_t)w1;
  return (uint32_t)__umul64hi(u, (uint64_t)n);
}

__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }
__device__ __forceinline__ double bitsd(uint64_t b) { return __longlong_as_double((long long)b); }

// log, positive normal finite x (fdlibm e_log.c reduction + polynomial)
__device__ __forceinline__ double plog(double x) {
  const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
  const double Lg1 = 0x1.5555555555593p-1, Lg2 = 0x1.999999997fa04p-2, Lg3 = 0x1.2492494229359p-2,
               Lg4 = 0x1.c71c51d8e78afp-3, Lg5 = 0x1.7466496cb03dep-3, Lg6 = 0x1.39a09d078c69fp-3,
               Lg7 = 0x1.2f112df3e5244p-3;
  uint64_t b = dbits(x);
  int k = (int)(b >> 52) - 1023;
  double m = bitsd((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
  bool big = m > 0x1.6a09e667f3bcdp+0;
  m = big ? m * 0.5 : m;
  k += big ? 1 : 0;
  double f = m - 1.0;
  double s = f / (2.0 + f);
  double dk = (double)k;
  double z = s * s;
  double w = z * z;
  double t1 = w * fma(w, fma(w, Lg6, Lg4), Lg2);
  double t2 = z * fma(w, fma(w, fma(w, Lg7, Lg5), Lg3), Lg1);
  double R = t2 + t1;
  double hfsq = 0.5 * f * f;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

// exp for x <= 0; 0 below -708
__device__ __forceinline__ double pexp(double x) {
  const double inv_ln2 = 0x1.71547652b82fep+0;
  const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
  bool tiny = !(x > -708.0);
  x = tiny ? 0.0 : x;
  double kd = floor(fma(x, inv_ln2, 0.5));
  double r = fma(-kd, ln2_hi, x);
  r = fma(-kd, ln2_lo, r);
  double p = 0x1.1eed8eff8d898p-29;
  p = fma(p, r, 0x1.ae64567f544e4p-26);
  p = fma(p, r, 0x1.27e4fb7789f5cp-22);
  p = fma(p, r, 0x1.71de3a556c734p-19);
  p = fma(p, r, 0x1.a01a01a01a01ap-16);
  p = fma(p, r, 0x1.a01a01a01a01ap-13);
  p = fma(p, r, 0x1.6c16c16c16c17p-10);
  p = fma(p, r, 0x1.1111111111111p-7);
  p = fma(p, r, 0x1.5555555555555p-5);
  p = fma(p, r, 0x1.5555555555555p-3);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  int k = (int)kd;
  double v = p * bitsd((uint64_t)(k + 1023) << 52);
  return tiny ? 0.0 : v;
}

// sqrt: bit-trick rsqrt seed, 4 Newton steps, one residual correction
__device__ __forceinline__ double psqrt(double a) {
  double y = bitsd(0x5FE6EB50C7B537A9ull - (dbits(a) >> 1));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double h = 0.5 * a * y;
    double e = fma(-h, y, 0.5);
    y = fma(y, e, y);
  }
  double r = a * y;
  double d = fma(-r, r, a);
  return fma(0.5 * y, d, r);
}

// sin/cos on |t| <= pi/4 (fdlibm kernel coefficients)
__device__ __forceinline__ void psincos(double t, double& s, double& c) {
  const double S1 = -0x1.5555555555549p-3, S2 = 0x1.111111110f8a6p-7, S3 = -0x1.a01a019c161d5p-13,
               S4 = 0x1.71de357b1fe7dp-19, S5 = -0x1.ae5e68a2b9cebp-26, S6 = 0x1.5d93a5acfd57cp-33;
  const double C1 = 0x1.555555555554cp-5, C2 = -0x1.6c16c16c15177p-10, C3 = 0x1.a01a019cb1590p-16,
               C4 = -0x1.27e4f809c52adp-22, C5 = 0x1.1ee9ebdb4b1c4p-29, C6 = -0x1.8fae9be8838d4p-37;
  double z = t * t;
  double ps = fma(z, S6, S5);
  ps = fma(z, ps, S4);
  ps = fma(z, ps, S3);
  ps = fma(z, ps, S2);
  ps = fma(z, ps, S1);
  double v = z * t;
  s = fma(v, ps, t);
  double pc = fma(z, C6, C5);
  pc = fma(z, pc, C4);
  pc = fma(z, pc, C3);
  pc = fma(z, pc, C2);
  pc = fma(z, pc, C1);
  double r = z * pc;
  double hz = 0.5 * z;
  double w = 1.0 - hz;
  c = w + (((1.0 - w) - hz) + z * r);
}

// Box-Muller pair from two words
__device__ __forceinline__ void normal_pair(uint32_t a, uint32_t b, double& z0, double& z1) {
  double u1 = ((double)a + 0.5) * 0x1p-32;
  double rho = psqrt(-2.0 * plog(u1));
  uint64_t bb = (uint64_t)b + 0x20000000ull;
  uint32_t q = (uint32_t)(bb >> 30) & 3u;
  int64_t ri = (int64_t)(bb & 0x3FFFFFFFull) - 0x20000000ll;
  double th = (((double)ri + 0.5) * 0x1p-30) * 0x1.921fb54442d18p+0;
  double s, c;
  psincos(th, s, c);
  double cs = (q & 1u) ? s : c;
  double sn = (q & 1u) ? c : s;
  cs = (q == 1u || q == 2u) ? -cs : cs;
  sn = (q >= 2u) ? -sn : sn;
  z0 = rho * cs;
  z1 = rho * sn;
}

// log1p(r), r in [0,1] (Goldberg: r * log(1+r) / ((1+r)-1)); log-sum-exp on the portable
// exp/log.  Drives the running nested-sampling estimate (nested.ml:139-142).
__device__ __forceinline__ double plog1p(double r) {
  double u = 1.0 + r;
  if (u == 1.0) return r;
  return plog(u) * (r / (u - 1.0));
}

__device__ __forceinline__ double plse(double a, double b) {
  if (a == -__builtin_inf() && b == -__builtin_inf()) return -__builtin_inf();
  if (b > a) {
    double t = a;
    a = b;
    b = t;
  }
  return a + plog1p(pexp(b - a));
}

// canonical 8-accumulator reduction tree (DESIGN.md §Canonical sums)
__device__ __forceinline__ double canon8(const double* A) {
  return ((A[0] + A[4]) + (A[2] + A[6])) + ((A[1] + A[5]) + (A[3] + A[7]));
}

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
  return __shfl_xor(v, m, 64);
}

}  // namespace mcg
