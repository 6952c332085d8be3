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

// log table (spec v2): {c_j, L_j} = {RN(128/(128+j)), RN(log(1+j/128))}, j = -38..53
__constant__ const double2 kLogTab[92] = {
  {0x1.6c16c16c16c17p+0, -0x1.68ac83e9c6a14p-2},  /* j = -38 */
  {0x1.6816816816817p+0, -0x1.5d5bddf595f30p-2},  /* j = -37 */
  {0x1.642c8590b2164p+0, -0x1.522ae0738a3d8p-2},  /* j = -36 */
  {0x1.6058160581606p+0, -0x1.4718dc271c41bp-2},  /* j = -35 */
  {0x1.5c9882b931057p+0, -0x1.3c25277333184p-2},  /* j = -34 */
  {0x1.58ed2308158edp+0, -0x1.314f1e1d35ce4p-2},  /* j = -33 */
  {0x1.5555555555555p+0, -0x1.269621134db92p-2},  /* j = -32 */
  {0x1.51d07eae2f815p+0, -0x1.1bf99635a6b95p-2},  /* j = -31 */
  {0x1.4e5e0a72f0539p+0, -0x1.1178e8227e47cp-2},  /* j = -30 */
  {0x1.4afd6a052bf5bp+0, -0x1.07138604d5862p-2},  /* j = -29 */
  {0x1.47ae147ae147bp+0, -0x1.f991c6cb3b379p-3},  /* j = -28 */
  {0x1.446f86562d9fbp+0, -0x1.e530effe71012p-3},  /* j = -27 */
  {0x1.4141414141414p+0, -0x1.d1037f2655e7bp-3},  /* j = -26 */
  {0x1.3e22cbce4a902p+0, -0x1.bd087383bd8adp-3},  /* j = -25 */
  {0x1.3b13b13b13b14p+0, -0x1.a93ed3c8ad9e3p-3},  /* j = -24 */
  {0x1.3813813813814p+0, -0x1.95a5adcf7017fp-3},  /* j = -23 */
  {0x1.3521cfb2b78c1p+0, -0x1.823c16551a3c2p-3},  /* j = -22 */
  {0x1.323e34a2b10bfp+0, -0x1.6f0128b756abcp-3},  /* j = -21 */
  {0x1.2f684bda12f68p+0, -0x1.5bf406b543db2p-3},  /* j = -20 */
  {0x1.2c9fb4d812ca0p+0, -0x1.4913d8333b561p-3},  /* j = -19 */
  {0x1.29e4129e4129ep+0, -0x1.365fcb0159016p-3},  /* j = -18 */
  {0x1.27350b8812735p+0, -0x1.23d712a49c202p-3},  /* j = -17 */
  {0x1.2492492492492p+0, -0x1.1178e8227e47cp-3},  /* j = -16 */
  {0x1.21fb78121fb78p+0, -0x1.fe89139dbd566p-4},  /* j = -15 */
  {0x1.1f7047dc11f70p+0, -0x1.da727638446a2p-4},  /* j = -14 */
  {0x1.1cf06ada2811dp+0, -0x1.b6ac88dad5b1cp-4},  /* j = -13 */
  {0x1.1a7b9611a7b96p+0, -0x1.9335e5d594989p-4},  /* j = -12 */
  {0x1.1811811811812p+0, -0x1.700d30aeac0e1p-4},  /* j = -11 */
  {0x1.15b1e5f75270dp+0, -0x1.4d3115d207eacp-4},  /* j = -10 */
  {0x1.135c81135c811p+0, -0x1.2aa04a44717a5p-4},  /* j = -9 */
  {0x1.1111111111111p+0, -0x1.08598b59e3a07p-4},  /* j = -8 */
  {0x1.0ecf56be69c90p+0, -0x1.ccb73cdddb2ccp-5},  /* j = -7 */
  {0x1.0c9714fbcda3bp+0, -0x1.894aa149fb343p-5},  /* j = -6 */
  {0x1.0a6810a6810a7p+0, -0x1.466aed42de3eap-5},  /* j = -5 */
  {0x1.0842108421084p+0, -0x1.0415d89e74444p-5},  /* j = -4 */
  {0x1.0624dd2f1a9fcp+0, -0x1.8492528c8cabfp-6},  /* j = -3 */
  {0x1.0410410410410p+0, -0x1.0205658935847p-6},  /* j = -2 */
  {0x1.0204081020408p+0, -0x1.010157588de71p-7},  /* j = -1 */
  {0x1.0000000000000p+0, 0x0.0p+0},  /* j = 0 */
  {0x1.fc07f01fc07f0p-1, 0x1.fe02a6b106789p-8},  /* j = 1 */
  {0x1.f81f81f81f820p-1, 0x1.fc0a8b0fc03e4p-7},  /* j = 2 */
  {0x1.f44659e4a4271p-1, 0x1.7b91b07d5b11bp-6},  /* j = 3 */
  {0x1.f07c1f07c1f08p-1, 0x1.f829b0e783300p-6},  /* j = 4 */
  {0x1.ecc07b301ecc0p-1, 0x1.39e87b9febd60p-5},  /* j = 5 */
  {0x1.e9131abf0b767p-1, 0x1.77458f632dcfcp-5},  /* j = 6 */
  {0x1.e573ac901e574p-1, 0x1.b42dd711971bfp-5},  /* j = 7 */
  {0x1.e1e1e1e1e1e1ep-1, 0x1.f0a30c01162a6p-5},  /* j = 8 */
  {0x1.de5d6e3f8868ap-1, 0x1.16536eea37ae1p-4},  /* j = 9 */
  {0x1.dae6076b981dbp-1, 0x1.341d7961bd1d1p-4},  /* j = 10 */
  {0x1.d77b654b82c34p-1, 0x1.51b073f06183fp-4},  /* j = 11 */
  {0x1.d41d41d41d41dp-1, 0x1.6f0d28ae56b4cp-4},  /* j = 12 */
  {0x1.d0cb58f6ec074p-1, 0x1.8c345d6319b21p-4},  /* j = 13 */
  {0x1.cd85689039b0bp-1, 0x1.a926d3a4ad563p-4},  /* j = 14 */
  {0x1.ca4b3055ee191p-1, 0x1.c5e548f5bc743p-4},  /* j = 15 */
  {0x1.c71c71c71c71cp-1, 0x1.e27076e2af2e6p-4},  /* j = 16 */
  {0x1.c3f8f01c3f8f0p-1, 0x1.fec9131dbeabbp-4},  /* j = 17 */
  {0x1.c0e070381c0e0p-1, 0x1.0d77e7cd08e59p-3},  /* j = 18 */
  {0x1.bdd2b899406f7p-1, 0x1.1b72ad52f67a0p-3},  /* j = 19 */
  {0x1.bacf914c1bad0p-1, 0x1.29552f81ff523p-3},  /* j = 20 */
  {0x1.b7d6c3dda338bp-1, 0x1.371fc201e8f74p-3},  /* j = 21 */
  {0x1.b4e81b4e81b4fp-1, 0x1.44d2b6ccb7d1ep-3},  /* j = 22 */
  {0x1.b2036406c80d9p-1, 0x1.526e5e3a1b438p-3},  /* j = 23 */
  {0x1.af286bca1af28p-1, 0x1.5ff3070a793d4p-3},  /* j = 24 */
  {0x1.ac5701ac5701bp-1, 0x1.6d60fe719d21dp-3},  /* j = 25 */
  {0x1.a98ef606a63bep-1, 0x1.7ab890210d909p-3},  /* j = 26 */
  {0x1.a6d01a6d01a6dp-1, 0x1.87fa06520c911p-3},  /* j = 27 */
  {0x1.a41a41a41a41ap-1, 0x1.9525a9cf456b4p-3},  /* j = 28 */
  {0x1.a16d3f97a4b02p-1, 0x1.a23bc1fe2b563p-3},  /* j = 29 */
  {0x1.9ec8e951033d9p-1, 0x1.af3c94e80bff3p-3},  /* j = 30 */
  {0x1.9c2d14ee4a102p-1, 0x1.bc286742d8cd6p-3},  /* j = 31 */
  {0x1.999999999999ap-1, 0x1.c8ff7c79a9a22p-3},  /* j = 32 */
  {0x1.970e4f80cb872p-1, 0x1.d5c216b4fbb91p-3},  /* j = 33 */
  {0x1.948b0fcd6e9e0p-1, 0x1.e27076e2af2e6p-3},  /* j = 34 */
  {0x1.920fb49d0e229p-1, 0x1.ef0adcbdc5936p-3},  /* j = 35 */
  {0x1.8f9c18f9c18fap-1, 0x1.fb9186d5e3e2bp-3},  /* j = 36 */
  {0x1.8d3018d3018d3p-1, 0x1.0402594b4d041p-2},  /* j = 37 */
  {0x1.8acb90f6bf3aap-1, 0x1.0a324e27390e3p-2},  /* j = 38 */
  {0x1.886e5f0abb04ap-1, 0x1.1058bf9ae4ad5p-2},  /* j = 39 */
  {0x1.8618618618618p-1, 0x1.1675cababa60ep-2},  /* j = 40 */
  {0x1.83c977ab2beddp-1, 0x1.1c898c16999fbp-2},  /* j = 41 */
  {0x1.8181818181818p-1, 0x1.22941fbcf7966p-2},  /* j = 42 */
  {0x1.7f405fd017f40p-1, 0x1.2895a13de86a3p-2},  /* j = 43 */
  {0x1.7d05f417d05f4p-1, 0x1.2e8e2bae11d31p-2},  /* j = 44 */
  {0x1.7ad2208e0ecc3p-1, 0x1.347dd9a987d55p-2},  /* j = 45 */
  {0x1.78a4c8178a4c8p-1, 0x1.3a64c556945eap-2},  /* j = 46 */
  {0x1.767dce434a9b1p-1, 0x1.404308686a7e4p-2},  /* j = 47 */
  {0x1.745d1745d1746p-1, 0x1.4618bc21c5ec2p-2},  /* j = 48 */
  {0x1.724287f46debcp-1, 0x1.4be5f957778a1p-2},  /* j = 49 */
  {0x1.702e05c0b8170p-1, 0x1.51aad872df82dp-2},  /* j = 50 */
  {0x1.6e1f76b4337c7p-1, 0x1.5767717455a6cp-2},  /* j = 51 */
  {0x1.6c16c16c16c17p-1, 0x1.5d1bdbf5809cap-2},  /* j = 52 */
  {0x1.6a13cd1537290p-1, 0x1.62c82f2b9c795p-2},  /* j = 53 */
};

// log for positive normal finite x (spec v2): fdlibm reduction to
// m in [sqrt(1/2), sqrt(2)), f = m - 1, j = round(128 f), r = (f - j/128) c_j, degree-7 log1p.
// `tab` points at kLogTab or at a copy staged in LDS (per-lane indices: an LDS gather).
__device__ __forceinline__ double plog(double x, const double2* tab) {
  const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
  const uint64_t b = dbits(x);
  int k = (int)(b >> 52) - 1023;
  double m = bitsd((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
  const bool big = m > 0x1.6a09e667f3bcdp+0;
  m = big ? m * 0.5 : m;
  k += big ? 1 : 0;
  const double f = m - 1.0;
  const double t = fma(f, 128.0, 0x1.8p52);
  const int j = (int)(uint32_t)dbits(t);
  const double jd = t - 0x1.8p52;
  const double d = fma(jd, -0x1p-7, f);
  const double2 cl = tab[j + 38];
  const double r = d * cl.x;
  const double z = r * r;
  double q = fma(r, 0x1.2492492492492p-3, -0x1.5555555555555p-3);
  q = fma(r, q, 0x1.999999999999ap-3);
  q = fma(r, q, -0.25);
  q = fma(r, q, 0x1.5555555555555p-2);
  q = fma(r, q, -0.5);
  const double p = fma(z, q, r);
  const double dk = (double)k;
  return fma(dk, ln2_hi, cl.y) + fma(dk, ln2_lo, p);
}

__device__ __forceinline__ double plog(double x) { return plog(x, kLogTab); }

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
  const double qc = fma(z, pc, -0.5);   // spec v3: cos = 1 + z (-1/2 + z P(z))
  c = fma(z, qc, 1.0);
}

// Box-Muller pair from two words
__device__ __forceinline__ void normal_pair(uint32_t a, uint32_t b, double& z0, double& z1,
                                            const double2* tab = kLogTab) {
  const double u1 = u32_open(a);
  const double rho = psqrt(-2.0 * plog(u1, tab));
  // quadrant q = round((b + 1/2) / 2^30) mod 4 and residual (ri + 1/2) 2^-30 in (-1/2, 1/2),
  // ri = ((b + 2^29) mod 2^30) - 2^29; the residual is built exactly from the 30 low bits:
  // (1 + u 2^-30) - (3/2 - 2^-31), u = (b + 2^29) mod 2^30.
  const uint32_t bb = b + 0x20000000u;
  const uint32_t q = (bb >> 30) & 3u;
  const uint32_t u = bb & 0x3FFFFFFFu;
  const double res = bitsd(((uint64_t)(0x3FF00000u | (u >> 10)) << 32) | (uint64_t)(u << 22)) -
                     (1.5 - 0x1p-31);
  const double th = res * 0x1.921fb54442d18p+0;
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
