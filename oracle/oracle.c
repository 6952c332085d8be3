/*
 * oracle.c -- CPU restatement of the farr/mcmc-ocaml hot path.  TEST INFRASTRUCTURE ONLY:
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER;
 * the product library (libmcg.so) never links or calls it.
 *
 * Parity status: see oracle.h.  Every function cites the reference file:line it restates
 * (paths relative to the farr/mcmc-ocaml root).  The randomness is injected: the OCaml stdlib
 * Random stream is replaced by the Philox4x32-10 stream specified in DESIGN.md §RNG, which the
 * HIP kernels draw identically, so GPU and oracle agree bit for bit.
 *
 * Build: oracle/Makefile  (gcc -O2 -ffp-contract=off; fma() is always explicit).
 */
#include "oracle.h"
#include "mcg.h"
#include "or_tables.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================================
 * RNG: Philox4x32-10 (Salmon et al. 2011) and variate conversions
 * ====================================================================================== */
#define PH_M0 0xD2511F53u
#define PH_M1 0xCD9E8D57u
#define PH_W0 0x9E3779B9u
#define PH_W1 0xBB67AE85u

void or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += PH_W0; k1 += PH_W1; }
    uint64_t p0 = (uint64_t)PH_M0 * c0;
    uint64_t p1 = (uint64_t)PH_M1 * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* counter layout: (c0, c1, c2, (tag << 16) | hi16) ; key = (seed_lo, seed_hi) */
#define TAG_MH 1u
#define TAG_NEST_WALK 3u
#define TAG_NEST_PRIOR 4u
#define TAG_POSTERIOR 5u
#define CALL_ACCEPT 0xFFFF0000u
#define CALL_DE_IDX 0xFFFF0001u
#define CALL_DE_SCALE 0xFFFF0002u
#define CALL_KD_PICK 0xFFFF0003u
#define CALL_START 0xFFFF0004u
#define CALL_MIX 0xFFFF0005u

static inline void rng4(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t tag,
                        uint32_t hi16, uint32_t out[4]) {
  uint32_t ctr[4] = {c0, c1, c2, (tag << 16) | (hi16 & 0xFFFFu)};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  or_philox(ctr, key, out);
}

/* uniform on (0,1): 52 random bits m -> (2m+1) 2^-53 */
double or_u53(uint32_t w0, uint32_t w1) {
  uint64_t m = ((uint64_t)w0 << 20) | (uint64_t)(w1 >> 12);
  return (double)((m << 1) | 1u) * 0x1p-53;
}

/* uniform integer in [0,n): floor(u64 * n / 2^64) */
uint32_t or_randint(uint32_t w0, uint32_t w1, uint32_t n) {
  uint64_t u = ((uint64_t)w0 << 32) | (uint64_t)w1;
  return (uint32_t)(((unsigned __int128)u * (unsigned __int128)n) >> 64);
}

/* ======================================================================================
 * Portable fp64 math: identical operation sequence on the device (csrc/mcg_math.h).
 * ====================================================================================== */
static inline uint64_t dbits(double x) { uint64_t b; memcpy(&b, &x, 8); return b; }
static inline double bitsd(uint64_t b) { double x; memcpy(&x, &b, 8); return x; }

/* log for positive normal finite x (spec v4, table-driven, division-free):
   x = 2^k m with the 52-bit mantissa rounded to 8 bits, j = round(256 (m - 1)) in [0, 256];
   cells j >= 106 are halved (m/2, k+1) so the reduced argument lies in [~0.707, ~1.414) and
   log x never cancels near x = 1.  With the cell centre m_j (exact bits),
   d = m - m_j is exact (Sterbenz), r = d * RN(1/m_j) (|r| <= 2^-9), and
   log x = k ln2 + log m_j + log1p(r), log1p by its degree-6 Taylor polynomial.
   Table: oracle/or_tables.h (oracle/gen_tables.py, mpmath). */
double or_log(double x) {
  const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
  uint64_t b = dbits(x);
  uint32_t hi = (uint32_t)(b >> 32), lo = (uint32_t)b;
  int k = (int)(hi >> 20) - 1023;
  uint32_t j = ((hi & 0xFFFFFu) + 0x800u) >> 12;                 /* 0..256 */
  int big = j >= OR_LOG_SPLIT;
  k += big;
  uint32_t mhi = (hi & 0xFFFFFu) | (big ? 0x3FE00000u : 0x3FF00000u);
  uint32_t chi = ((0x3FF00u + j) << 12) - (big ? 0x100000u : 0u);
  double m = bitsd(((uint64_t)mhi << 32) | lo);
  double mj = bitsd((uint64_t)chi << 32);
  double d = m - mj;
  double r = d * or_logtab[j][0];
  double z = r * r;
  double q = fma(r, -0x1.5555555555555p-3, 0x1.999999999999ap-3);   /* -1/6, 1/5 */
  q = fma(r, q, -0.25);
  q = fma(r, q, 0x1.5555555555555p-2);                                /* 1/3 */
  q = fma(r, q, -0.5);
  double p = fma(z, q, r);
  double dk = (double)k;
  return fma(dk, ln2_hi, or_logtab[j][1]) + fma(dk, ln2_lo, p);
}

/* exp for x <= 0 (used by log-space accumulators); returns 0 below -708, 1 at 0. */
double or_exp(double x) {
  if (!(x > -708.0)) return 0.0;   /* also NaN -> 0 is never reached by callers */
  const double inv_ln2 = 0x1.71547652b82fep+0;
  const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
  double kd = floor(fma(x, inv_ln2, 0.5));
  double r = fma(-kd, ln2_hi, x);
  r = fma(-kd, ln2_lo, r);
  double p = 0x1.1eed8eff8d898p-29;          /* 1/12! */
  p = fma(p, r, 0x1.ae64567f544e4p-26);      /* 1/11! */
  p = fma(p, r, 0x1.27e4fb7789f5cp-22);      /* 1/10! */
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
  return p * bitsd((uint64_t)(k + 1023) << 52);
}

/* sqrt (spec v3): bit-trick rsqrt seed, 4 Newton steps on 1/sqrt(a), then a * y (<= 2 ulp) */
double or_sqrt(double a) {
  double y = bitsd(0x5FE6EB50C7B537A9ull - (dbits(a) >> 1));
  double ha = 0.5 * a;
  for (int i = 0; i < 4; ++i) {
    double h = ha * y;
    double e = fma(-h, y, 0.5);
    y = fma(y, e, y);
  }
  return a * y;
}

/* standard normal from one 32-bit word (spec v7): z = -+ q(u), the sign from bit 31, u = v 2^-33
   with v = 2 (w mod 2^31) + 1, and q the spec's piecewise-polynomial normal quantile on (0, 1/2):
   for v = 2^E (1 + f), segment (E, j = floor(32 f)), t = 32 f - j in [0, 1), Horner (fma) in
   x' = 1 + t/32 of the segment's four coefficients (or_tables.h, highest first).  Replaces
   Leva's ratio-of-uniforms Stats.draw_gaussian (stats.ml:113-124): any exactly symmetric
   proposal keeps MH exact, and the table is within 7.5e-10 of the exact quantile (about one
   step of the grid the 2^-32 quantisation of u puts on z). */
double or_normal(uint32_t w) {
  uint32_t v = 2u * (w & 0x7FFFFFFFu) + 1u;
  int E = 31 - __builtin_clz(v);
  double fv = ldexp((double)v, -E);                /* exact, in [1, 2) */
  int j = (int)((fv - 1.0) * 32.0);                /* exact product, then floor */
  double xp = fv - ldexp((double)j, -5);           /* exact: 1 + t/32 */
  const double(*c)[2] = &or_nrmtab[2 * (E * 32 + j)];
  double p = fma(c[0][0], xp, c[0][1]);
  p = fma(p, xp, c[1][0]);
  p = fma(p, xp, c[1][1]);
  return (w >> 31) ? -p : p;
}

/* log1p(r) for r in [0,1] and log-sum-exp with the portable exp/log (device-reproducible):
   log1p(r) = r * log(1+r) / ((1+r) - 1) (Goldberg); used for the running nested-sampling
   estimate that drives the stopping rule (nested.ml:139-142). */
double or_plog1p(double r) {
  double u = 1.0 + r;
  if (u == 1.0) return r;
  return or_log(u) * (r / (u - 1.0));
}

double or_plse(double a, double b) {
  if (a == -INFINITY && b == -INFINITY) return -INFINITY;
  if (b > a) { double t = a; a = b; b = t; }
  return a + or_plog1p(or_exp(b - a));
}

/* dims 4c..4c+3 of a step take Philox call c: word k -> z[4c + k] */
static void normals_tagged(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t tag, uint32_t hi16,
                           int D, double* z) {
  for (int c = 0; 4 * c < D; ++c) {
    uint32_t w[4];
    rng4(seed, c0, c1, (uint32_t)c, tag, hi16, w);
    for (int j = 0; j < 4 && 4 * c + j < D; ++j) z[4 * c + j] = or_normal(w[j]);
  }
}

void or_step_normals(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, int D, double* z) {
  normals_tagged(seed, chain, (uint32_t)step, tag, (uint32_t)(step >> 32), D, z);
}

/* ======================================================================================
 * Stats restatements (stats.ml)
 * ====================================================================================== */
double or_log_sum_logs(double a, double b) {      /* stats.ml:240-248 */
  if (a == -INFINITY && b == -INFINITY) return -INFINITY;
  if (b > a) { double t = a; a = b; b = t; }
  return a + log1p(exp(b - a));
}

double or_mean(const double* xs, int64_t n) {     /* stats.ml:17-23 */
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s = s + xs[i];
  return s / (double)n;
}

double or_std(const double* xs, int64_t n) {      /* stats.ml:35-43 */
  double mu = or_mean(xs, n), v = 0.0;
  for (int64_t i = 0; i < n; ++i) { double x = xs[i] - mu; v = v + x * x; }
  return sqrt(v / (double)(n - 1));
}

void or_multi_mean(const double* xs, int64_t n, int d, double* mu) {   /* stats.ml:58-70 */
  for (int j = 0; j < d; ++j) mu[j] = 0.0;
  for (int64_t i = 0; i < n; ++i)
    for (int j = 0; j < d; ++j) mu[j] = mu[j] + xs[i * d + j];
  for (int j = 0; j < d; ++j) mu[j] = mu[j] / (double)n;
}

void or_multi_std(const double* xs, int64_t n, int d, double* sd) {    /* stats.ml:72-87 */
  double* mu = (double*)malloc(sizeof(double) * (size_t)d);
  or_multi_mean(xs, n, d, mu);
  for (int j = 0; j < d; ++j) sd[j] = 0.0;
  for (int64_t i = 0; i < n; ++i)
    for (int j = 0; j < d; ++j) { double dx = xs[i * d + j] - mu[j]; sd[j] = sd[j] + dx * dx; }
  for (int j = 0; j < d; ++j) sd[j] = sqrt(sd[j] / (double)(n - 1));
  free(mu);
}

static const double NEG_HALF_LOG_2PI = -0.91893853320467274178;
static const double OR_PI = 3.14159265358979323846;

double or_log_gaussian(double mu, double sigma, double x) {            /* stats.ml:98-101 */
  double dx = (x - mu) / sigma;
  return NEG_HALF_LOG_2PI - log(sigma) - 0.5 * dx * dx;
}

double or_log_cauchy(double x0, double gamma, double x) {             /* stats.ml:93-96 */
  double dx = (x - x0) / gamma;
  return 0.0 - log(OR_PI * gamma) - log(1.0 + dx * dx);
}

double or_log_multi_gaussian(const double* mu, const double* sigma, const double* x, int d) {
  double r = 0.0;                                                      /* stats.ml:103-108 */
  for (int i = 0; i < d; ++i) r = r + or_log_gaussian(mu[i], sigma[i], x[i]);
  return r + 0.0;
}

double or_log_lognormal(double mu, double sigma, double x) {          /* stats.ml:217-221 */
  double lx = log(x), d = (lx - mu) / sigma, ls = log(sigma);
  return NEG_HALF_LOG_2PI - lx - ls - 0.5 * d * d;
}

/* ======================================================================================
 * Model preparation (host-side constants shared with libmcg's mcg_set_* semantics)
 * ====================================================================================== */
typedef struct {
  int D, lik, prior, prop;
  double* mu; double* isig; double C;          /* DIAG_GAUSS / FULLCOV (mu) */
  const double* U;                             /* FULLCOV */
  double* ctr; double R, iw;                   /* SHELL */
  int nd; int64_t nsamp; const double* data;   /* GAUSS_DATA / CAUCHY_DATA */
  const double* lo; const double* hi; double lp_in;   /* BOX priors */
  double* s;                                   /* GAUSS proposal scales [D] */
  const double* wlo; const double* whi; const double* wdx;   /* WRAP_UNIFORM */
  const or_kd* kd;
  int nmix; struct mix_comp* mix; int mix_kd;  /* MIXTURE (combine_jump_proposals) */
  double de_mh, de_sigma; int64_t de_M; const double* de_pts;   /* DE: samples [M][D] */
  const double* raw_lik;                       /* the caller's likelihood parameters */
  int ngm; double* gm;                         /* GAUSS_MIX: per component mu/s[D], 1/s[D], C */
  double* gp; const double* gp_mu; const double* gp_sig;   /* DIAG_GAUSS prior: mu/s[D], 1/s[D], C */
} prep_t;

/* one component of Mcmc.combine_jump_proposals (mcmc.ml:165-185): normalised weight p, log p,
   kind (MCG_MIX_*), ljp mode (0: log_jump_prob = 0, 1: the component's log density) */
struct mix_comp {
  double p, logp, C;
  int kind, mode;
  const double* v0; const double* v1; const double* v2;   /* GAUSS: s; SHIFT: a, b; WRAP: lo, hi, dx */
  double* inv_s;                                           /* GAUSS: 1/s */
  double* width;                                           /* SHIFT: b - a */
};

static void prep_free(prep_t* p) {
  free(p->mu); free(p->isig); free(p->ctr); free(p->s); free(p->gm); free(p->gp);
  if (p->mix)
    for (int c = 0; c < p->nmix; ++c) { free(p->mix[c].inv_s); free(p->mix[c].width); }
  free(p->mix);
}

static int prep_model_(const or_model* m, prep_t* p);

/* the model's constants; on invalid parameters everything allocated so far is freed */
static int prep_model(const or_model* m, prep_t* p) {
  const int rc = prep_model_(m, p);
  if (rc != 0) {
    prep_free(p);
    memset(p, 0, sizeof(*p));
  }
  return rc;
}

static int prep_model_(const or_model* m, prep_t* p) {
  memset(p, 0, sizeof(*p));
  int D = m->ndim;
  p->D = D; p->lik = m->lik_kind; p->prior = m->prior_kind; p->prop = m->prop_kind;
  const double* q = m->lik_params;
  p->raw_lik = q;
  switch (p->lik) {
    case MCG_LIK_FLAT: break;
    case MCG_LIK_DIAG_GAUSS:
      /* constants: 1/sigma_d, mu_d/sigma_d (= RN(mu_d * RN(1/sigma_d))), C */
      p->mu = (double*)malloc(sizeof(double) * D);
      p->isig = (double*)malloc(sizeof(double) * D);
      p->C = 0.0;
      for (int d = 0; d < D; ++d) {
        p->isig[d] = 1.0 / q[D + d];
        p->mu[d] = q[d] * p->isig[d];
        p->C = p->C + (NEG_HALF_LOG_2PI - log(q[D + d]));
      }
      break;
    case MCG_LIK_FULLCOV_GAUSS:
      p->mu = (double*)malloc(sizeof(double) * D);
      for (int d = 0; d < D; ++d) p->mu[d] = q[d];
      p->U = q + D;
      p->C = 0.0;
      for (int i = 0; i < D; ++i) p->C = p->C + (log(p->U[i * D + i]) + NEG_HALF_LOG_2PI);
      break;
    case MCG_LIK_GAUSS_SHELL:
      p->ctr = (double*)malloc(sizeof(double) * D);
      for (int d = 0; d < D; ++d) p->ctr[d] = q[d];
      p->R = q[D];
      p->iw = 1.0 / q[D + 1];
      p->C = NEG_HALF_LOG_2PI - log(q[D + 1]);
      break;
    case MCG_LIK_GAUSS_DATA:
    case MCG_LIK_CAUCHY_DATA:
      p->nd = (int)q[0];
      p->data = q + 1;
      p->nsamp = (m->n_lik_params - 1) / p->nd;
      break;
    case MCG_LIK_GAUSS_MIX:
      /* m, then per component mu[D], sigma[D]; each component's DIAG constants as above */
      p->ngm = (int)q[0];
      if (p->ngm < 1 || p->ngm > MCG_LIK_MIX_MAX || m->n_lik_params != 1 + (int64_t)p->ngm * 2 * D) return -1;
      p->gm = (double*)malloc(sizeof(double) * (size_t)p->ngm * (2 * D + 1));
      for (int c = 0; c < p->ngm; ++c) {
        const double* mu = q + 1 + (size_t)c * 2 * D;
        double* o = p->gm + (size_t)c * (2 * D + 1);
        double C = 0.0;
        for (int d = 0; d < D; ++d) {
          o[D + d] = 1.0 / mu[D + d];
          o[d] = mu[d] * o[D + d];
          C = C + (NEG_HALF_LOG_2PI - log(mu[D + d]));
        }
        o[2 * D] = C;
      }
      break;
    default: return -1;
  }
  if (p->prior == MCG_PRIOR_BOX || p->prior == MCG_PRIOR_OPEN_BOX) {
    p->lo = m->prior_params; p->hi = m->prior_params + D; p->lp_in = m->prior_params[2 * D];
  } else if (p->prior == MCG_PRIOR_DIAG_GAUSS) {
    /* Stats.log_multi_gaussian mu sigma as a log_prior (stats.ml:98-108): the DIAG_GAUSS
       likelihood's canonical constants (above) of the prior's mu, sigma */
    const double* pq = m->prior_params;
    if (m->n_prior_params != 2 * (int64_t)D) return -1;
    p->gp_mu = pq; p->gp_sig = pq + D;
    p->gp = (double*)malloc(sizeof(double) * (size_t)(2 * D + 1));
    double C = 0.0;
    for (int d = 0; d < D; ++d) {
      if (!(pq[D + d] > 0.0)) return -1;
      p->gp[D + d] = 1.0 / pq[D + d];
      p->gp[d] = pq[d] * p->gp[D + d];
      C = C + (NEG_HALF_LOG_2PI - log(pq[D + d]));
    }
    p->gp[2 * D] = C;
  }
  if (p->prop == MCG_PROP_GAUSS) {
    p->s = (double*)malloc(sizeof(double) * D);
    for (int d = 0; d < D; ++d) p->s[d] = (m->n_prop_params == 1) ? m->prop_params[0] : m->prop_params[d];
  } else if (p->prop == MCG_PROP_WRAP_UNIFORM) {
    p->wlo = m->prop_params; p->whi = m->prop_params + D; p->wdx = m->prop_params + 2 * D;
  } else if (p->prop == MCG_PROP_KD_INTERP) {
    p->kd = (const or_kd*)m->kd;
  } else if (p->prop == MCG_PROP_DE) {
    /* oracle parameters: mode_hopping_frac, M, samples [M][D]; sigma of mcmc.ml:212 */
    if (m->n_prop_params < 2) return -1;
    p->de_mh = m->prop_params[0];
    p->de_M = (int64_t)m->prop_params[1];
    p->de_pts = m->prop_params + 2;
    if (p->de_M < 2 || m->n_prop_params != 2 + p->de_M * D) return -1;
    p->de_sigma = 2.38 / sqrt(2.0 * (double)D);
  } else if (p->prop == MCG_PROP_MIXTURE) {
    /* parameters: ncomp, then per component p, kind, ljp_mode, params (include/mcg.h) */
    const double* q = m->prop_params;
    int nc = (int)q[0];
    if (nc < 1 || nc > MCG_MIX_MAX_COMPONENTS) return -1;
    p->nmix = nc;
    p->mix = (struct mix_comp*)calloc((size_t)nc, sizeof(struct mix_comp));
    p->kd = (const or_kd*)m->kd;
    double ptot = 0.0;
    int64_t o = 1;
    for (int c = 0; c < nc; ++c) {
      struct mix_comp* mc = &p->mix[c];
      mc->p = q[o]; mc->kind = (int)q[o + 1]; mc->mode = (int)q[o + 2];
      const double* u = q + o + 3;
      ptot = ptot + mc->p;                                   /* mcmc.ml:166 */
      switch (mc->kind) {
        case MCG_MIX_GAUSS:
          mc->v0 = u;
          mc->inv_s = (double*)malloc(sizeof(double) * D);
          mc->C = 0.0;
          for (int d = 0; d < D; ++d) {
            mc->inv_s[d] = 1.0 / u[d];
            mc->C = mc->C + (NEG_HALF_LOG_2PI - log(u[d]));
          }
          o += 3 + D;
          break;
        case MCG_MIX_SHIFT_UNIFORM:
          mc->v0 = u; mc->v1 = u + D;
          mc->width = (double*)malloc(sizeof(double) * D);
          mc->C = 0.0;
          for (int d = 0; d < D; ++d) {
            mc->width[d] = u[D + d] - u[d];
            mc->C = mc->C - log(mc->width[d]);
          }
          o += 3 + 2 * D;
          break;
        case MCG_MIX_WRAP_UNIFORM:
          mc->v0 = u; mc->v1 = u + D; mc->v2 = u + 2 * D;
          o += 3 + 3 * D;
          break;
        case MCG_MIX_KD_INTERP:
          mc->mode = 1;
          p->mix_kd = 1;
          if (!p->kd) return -1;
          o += 3;
          break;
        default: return -1;
      }
    }
    for (int c = 0; c < nc; ++c) {
      p->mix[c].p = p->mix[c].p / ptot;                     /* mcmc.ml:167 */
      p->mix[c].logp = log(p->mix[c].p);
    }
  }
  return 0;
}

/* canonical 8-accumulator sum: term of dim d goes to A[(d>>2)&7] (sequential in d), then
   S = ((A0+A4)+(A2+A6)) + ((A1+A5)+(A3+A7)).  Independent of how many lanes share a chain. */
static inline double canon8(const double* A) {
  return ((A[0] + A[4]) + (A[2] + A[6])) + ((A[1] + A[5]) + (A[3] + A[7]));
}

/* ---- the reference's literal arithmetic (DESIGN.md §2 "literal mode") ----
 * The canonical arithmetic above (fma residuals, 8-accumulator sum, host constant C, portable
 * log of the accept uniform, portable log-sum of the nested running estimate) is what the GPU
 * computes.  or_set_literal(1) switches the oracle to the reference's own operation order:
 * Stats.log_multi_gaussian (stats.ml:98-108: division, sequential sum from d = 0, glibc log sigma
 * in every term, the trailing +. 0.0), glibc log of the accept uniform (mcmc.ml:49), and
 * Stats.log_sum_logs with glibc exp / log1p (stats.ml:240-248) for the nested running estimate
 * and stop test, folded one retired point at a time (nested.ml:138-141).  The Gaussian shell
 * (no reference closure) is Stats.log_gaussian of the sequential-sum radius.  Process-wide;
 * set it before a run, not during one. */
static int g_literal = 0;
void or_set_literal(int on) { g_literal = on != 0; }
int or_get_literal(void) { return g_literal; }

static double lik_literal(const prep_t* p, const double* x) {
  const int D = p->D;
  const double* q = p->raw_lik;
  if (p->lik == MCG_LIK_DIAG_GAUSS) {
    double result = 0.0;
    for (int i = 0; i < D; ++i) {
      double dx = (x[i] - q[i]) / q[D + i];
      result = result + ((-0.91893853320467274178 - log(q[D + i])) - 0.5 * dx * dx);
    }
    return result + 0.0;
  }
  if (p->lik == MCG_LIK_GAUSS_SHELL) {
    double ss = 0.0;
    for (int i = 0; i < D; ++i) { double e = x[i] - q[i]; ss = ss + e * e; }
    double dx = (sqrt(ss) - q[D]) / q[D + 1];
    return (-0.91893853320467274178 - log(q[D + 1])) - 0.5 * dx * dx;
  }
  if (p->lik == MCG_LIK_GAUSS_MIX) {
    /* test/nested_test.ml:52-57: log ((exp g1) +. (exp g2) +. ...), left to right, each g_i
       Stats.log_multi_gaussian mu_i sigma_i x (stats.ml:103-108) */
    double sum = 0.0;
    for (int c = 0; c < p->ngm; ++c) {
      const double* mu = q + 1 + (size_t)c * 2 * D;
      const double* sg = mu + D;
      double result = 0.0;
      for (int i = 0; i < D; ++i) {
        double dx = (x[i] - mu[i]) / sg[i];
        result = result + ((-0.91893853320467274178 - log(sg[i])) - 0.5 * dx * dx);
      }
      const double e = exp(result + 0.0);
      sum = c == 0 ? e : sum + e;
    }
    return log(sum);
  }
  return NAN;
}

static double lik_eval(const prep_t* p, const double* x) {
  int D = p->D;
  if (g_literal && (p->lik == MCG_LIK_DIAG_GAUSS || p->lik == MCG_LIK_GAUSS_SHELL || p->lik == MCG_LIK_GAUSS_MIX))
    return lik_literal(p, x);
  double A[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  switch (p->lik) {
    case MCG_LIK_FLAT: return 0.0;
    case MCG_LIK_DIAG_GAUSS: {
      for (int d = 0; d < D; ++d) {
        double e = fma(x[d], p->isig[d], -p->mu[d]);     /* (x - mu)/sigma as x/s - mu/s */
        A[(d >> 2) & 7] = fma(e, e, A[(d >> 2) & 7]);
      }
      return p->C - 0.5 * canon8(A);
    }
    case MCG_LIK_FULLCOV_GAUSS: {
      double r[256];
      for (int d = 0; d < D; ++d) r[d] = x[d] - p->mu[d];
      for (int i = 0; i < D; ++i) {
        double t = 0.0;
        for (int j = i; j < D; ++j) t = fma(p->U[i * D + j], r[j], t);
        /* FULLCOV accumulator of row i: (i & 3) | ((i >> 4) & 1) << 2 -- the rows a lane
           quadrant of the MFMA output holds (csrc/mcg_fullcov_kernel.h) */
        int k = (i & 3) | (((i >> 4) & 1) << 2);
        A[k] = fma(t, t, A[k]);
      }
      return p->C - 0.5 * canon8(A);
    }
    case MCG_LIK_GAUSS_MIX: {
      /* canonical: each component's DIAG canonical sum, folded by a one-pass max-shifted
         log-sum-exp in component order (csrc/mcg_mh_kernel.h eval_lik) */
      double M = -INFINITY, sacc = 0.0;
      for (int c = 0; c < p->ngm; ++c) {
        const double* qc = p->gm + (size_t)c * (2 * D + 1);
        double B[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int d = 0; d < D; ++d) {
          double e = fma(x[d], qc[D + d], -qc[d]);
          B[(d >> 2) & 7] = fma(e, e, B[(d >> 2) & 7]);
        }
        const double g = qc[2 * D] - 0.5 * canon8(B);
        if (g > M) {
          sacc = sacc * or_exp(M - g) + 1.0;
          M = g;
        } else {
          sacc = sacc + or_exp(g - M);
        }
      }
      return M == -INFINITY ? M : M + or_log(sacc);
    }
    case MCG_LIK_GAUSS_SHELL: {
      for (int d = 0; d < D; ++d) {
        double e = x[d] - p->ctr[d];
        A[(d >> 2) & 7] = fma(e, e, A[(d >> 2) & 7]);
      }
      double r = or_sqrt(canon8(A));
      double qq = (r - p->R) * p->iw;
      return p->C - 0.5 * qq * qq;
    }
    case MCG_LIK_GAUSS_DATA:
    case MCG_LIK_CAUCHY_DATA: {
      /* bin/gaussian_cauchy.ml:149-164: sum_i sum_j prob mu_j sigma_j samp_ij */
      int nd = p->nd;
      const double* mu = x;
      const double* sg = x + nd;
      double lterm[64];
      for (int j = 0; j < nd; ++j)
        lterm[j] = (p->lik == MCG_LIK_GAUSS_DATA) ? or_log(sg[j]) : or_log(OR_PI * sg[j]);
      double acc = 0.0;
      for (int64_t i = 0; i < p->nsamp; ++i) {
        for (int j = 0; j < nd; ++j) {
          double dx = (p->data[i * nd + j] - mu[j]) / sg[j];
          double term;
          if (p->lik == MCG_LIK_GAUSS_DATA)
            term = (NEG_HALF_LOG_2PI - lterm[j]) - 0.5 * dx * dx;     /* stats.ml:98-101 */
          else
            term = (0.0 - lterm[j]) - or_log(1.0 + dx * dx);          /* stats.ml:93-96 */
          acc = acc + term;
        }
      }
      return acc + 0.0;
    }
  }
  return NAN;
}

static double prior_eval(const prep_t* p, const double* x) {
  if (p->prior == MCG_PRIOR_FLAT) return 0.0;
  if (p->prior == MCG_PRIOR_DIAG_GAUSS) {
    if (g_literal) return or_log_multi_gaussian(p->gp_mu, p->gp_sig, x, p->D);   /* stats.ml:103-108 */
    double A[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int d = 0; d < p->D; ++d) {
      double e = fma(x[d], p->gp[p->D + d], -p->gp[d]);
      A[(d >> 2) & 7] = fma(e, e, A[(d >> 2) & 7]);
    }
    return p->gp[2 * p->D] - 0.5 * canon8(A);
  }
  int inb = 1;
  for (int d = 0; d < p->D; ++d) {
    if (p->prior == MCG_PRIOR_BOX) inb &= (x[d] >= p->lo[d]) & (x[d] <= p->hi[d]);
    else inb &= (x[d] > p->lo[d]) & (x[d] < p->hi[d]);
  }
  return inb ? p->lp_in : -INFINITY;
}

double or_loglik(const or_model* m, const double* x) {
  prep_t p; prep_model(m, &p); double v = lik_eval(&p, x); prep_free(&p); return v;
}
double or_logprior(const or_model* m, const double* x) {
  prep_t p; prep_model(m, &p); double v = prior_eval(&p, x); prep_free(&p); return v;
}

/* Mcmc.uniform_wrapping (mcmc.ml:187-196) with the uniform injected: the reference's loop
 * (mcmc.ml:189-195) exactly for up to OR_WRAP_EXACT reflections; an exit where that loop never
 * ends (nx == xmax reflects onto itself; rounding 2-cycles at |nx| >> width); past the bound the
 * remaining excess folded by the loop's real-arithmetic limit (triangle wave of period 2w). */
#define OR_WRAP_EXACT 1024
double or_wrap_uniform(double xmin, double xmax, double dx, double x, double u) {
  double nx = x + (u - 0.5) * dx;
  for (int it = 0; it < OR_WRAP_EXACT; ++it) {
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
#define wrap_uniform or_wrap_uniform

/* ======================================================================================
 * kD tree (kd_tree.ml) + Interpolate_pdf (interpolate_pdf.ml) -- declared here, defined below
 * ====================================================================================== */
struct or_kd {
  int D; int64_t M;
  int64_t nn, nl, cap_n, cap_l;
  int32_t* dim; double* split; int32_t* right; int32_t* leaf;
  int32_t* lcount; double* lbox; double* llogq;
  double* root_lo; double* root_hi;
  double* pts;                               /* copy of the M training points [M][D] */
};

static int64_t kd_find_leaf_idx(const or_kd* t, const double* pt);

/* ======================================================================================
 * One MH step (mcmc.ml:37-56) for one chain, RNG injected
 * ====================================================================================== */
typedef struct {
  double x[256]; double ll, lp; double lq;   /* lq: cached log q(x) for KD_INTERP */
} chain_t;

/* Mcmc.log_sum_logs, the private one of mcmc.ml:155-163: log (1 + exp lr) */
static double mix_lse(double la, double lb) {
  if (la == -INFINITY && lb == -INFINITY) return -INFINITY;
  if (la > lb) return la + or_log(1.0 + or_exp(lb - la));
  return lb + or_log(1.0 + or_exp(la - lb));
}

/* log_jp x y of combine_jump_proposals (mcmc.ml:175-182), lq_y = log q(y) of the kD tree */
static double mix_log_jp(const prep_t* p, const double* x, const double* y, double lq_y) {
  int D = p->D;
  double acc = -INFINITY;
  for (int c = 0; c < p->nmix; ++c) {
    const struct mix_comp* mc = &p->mix[c];
    double lj = 0.0;
    if (mc->mode) {
      if (mc->kind == MCG_MIX_GAUSS) {
        double S = 0.0;
        for (int d = 0; d < D; ++d) {
          double e = (y[d] - x[d]) * mc->inv_s[d];
          S = fma(e, e, S);
        }
        lj = mc->C - 0.5 * S;
      } else if (mc->kind == MCG_MIX_SHIFT_UNIFORM) {
        int in = 1;   /* test/mcmc_test.ml:188-197: y >= x + a && y <= x + b */
        for (int d = 0; d < D; ++d) in = in && y[d] >= x[d] + mc->v0[d] && y[d] <= x[d] + mc->v1[d];
        lj = in ? mc->C : -INFINITY;
      } else if (mc->kind == MCG_MIX_KD_INTERP) {
        lj = lq_y;
      }
    }
    acc = mix_lse(acc, mc->logp + lj);
  }
  return acc;
}

typedef struct { double y[256]; double lly, lpy, ratio, u; int acc; } step_probe;

static int mh_step(const prep_t* p, uint64_t seed, uint32_t gid, uint64_t T, chain_t* c,
                   step_probe* pr) {
  int D = p->D;
  uint32_t lo = (uint32_t)T, hi = (uint32_t)(T >> 32);
  double y[256];
  double lf = 0.0, lb = 0.0, lqy = 0.0;
  switch (p->prop) {
    case MCG_PROP_GAUSS: {
      double z[256];
      normals_tagged(seed, gid, lo, TAG_MH, hi, D, z);
      for (int d = 0; d < D; ++d) y[d] = fma(p->s[d], z[d], c->x[d]);
      break;
    }
    case MCG_PROP_WRAP_UNIFORM: {
      for (int d = 0; d < D; d += 2) {
        uint32_t w[4];
        rng4(seed, gid, lo, (uint32_t)(d >> 1), TAG_MH, hi, w);
        y[d] = wrap_uniform(p->wlo[d], p->whi[d], p->wdx[d], c->x[d], or_u53(w[0], w[1]));
        if (d + 1 < D)
          y[d + 1] = wrap_uniform(p->wlo[d + 1], p->whi[d + 1], p->wdx[d + 1], c->x[d + 1],
                                  or_u53(w[2], w[3]));
      }
      break;
    }
    case MCG_PROP_KD_INTERP: {
      /* Interpolate_pdf.draw (interpolate_pdf.ml:114-119): pick a training point, find its
         leaf, draw uniformly in the leaf box. */
      const or_kd* t = p->kd;
      uint32_t w[4];
      rng4(seed, gid, lo, CALL_KD_PICK, TAG_MH, hi, w);
      uint32_t pick = or_randint(w[0], w[1], (uint32_t)t->M);
      const double* pt = t->pts + (int64_t)pick * D;
      int64_t L = kd_find_leaf_idx(t, pt);
      const double* blo = t->lbox + L * 2 * D;
      const double* bhi = blo + D;
      for (int d = 0; d < D; d += 2) {
        rng4(seed, gid, lo, (uint32_t)(d >> 1), TAG_MH, hi, w);
        y[d] = blo[d] + (bhi[d] - blo[d]) * or_u53(w[0], w[1]);
        if (d + 1 < D) y[d + 1] = blo[d + 1] + (bhi[d + 1] - blo[d + 1]) * or_u53(w[2], w[3]);
      }
      lqy = t->llogq[kd_find_leaf_idx(t, y)];
      lf = lqy;         /* log_jump_prob start proposed = log q(proposed) */
      lb = c->lq;       /* log_jump_prob proposed start = log q(start) */
      break;
    }
    case MCG_PROP_DE: {
      /* Mcmc.differential_evolution_proposal (mcmc.ml:198-218): pick_samples i != j
         (:199-203; j from the n - 1 others instead of the retry loop), d = 1.0 with
         probability mode_hopping_frac (:209; the && short-circuits at 0) else
         draw_gaussian 0.0 sigma (:212-213), z'_d = z_d + d (y_d - x_d) (:214-217) */
      uint32_t w[4];
      rng4(seed, gid, lo, CALL_DE_IDX, TAG_MH, hi, w);
      uint32_t n = (uint32_t)p->de_M;
      uint32_t i = or_randint(w[0], w[1], n);
      uint32_t jj = or_randint(w[2], w[3], n - 1);
      uint32_t j = jj + (jj >= i ? 1u : 0u);
      rng4(seed, gid, lo, CALL_DE_SCALE, TAG_MH, hi, w);
      double dsc;
      if (p->de_mh != 0.0 && or_u53(w[0], w[1]) < p->de_mh) dsc = 1.0;
      else dsc = p->de_sigma * or_normal(w[2]);
      const double* xi = p->de_pts + (int64_t)i * D;
      const double* yj = p->de_pts + (int64_t)j * D;
      for (int d = 0; d < D; ++d) y[d] = c->x[d] + dsc * (yj[d] - xi[d]);
      break;
    }
    case MCG_PROP_MIXTURE: {
      /* propose: Random.float 1.0 walked down the normalised weights (mcmc.ml:168-173); the
         reference raises Failure past the last weight (:173) -- the product refuses such weights at
         configuration (pack_mixture); the walk here keeps the last component */
      uint32_t w[4];
      rng4(seed, gid, lo, CALL_MIX, TAG_MH, hi, w);
      double u = or_u53(w[0], w[1]);
      int pick = p->nmix - 1;
      for (int k = 0; k < p->nmix; ++k) {
        if (u < p->mix[k].p) { pick = k; break; }
        u = u - p->mix[k].p;
      }
      const struct mix_comp* mc = &p->mix[pick];
      if (mc->kind == MCG_MIX_GAUSS) {
        double z[256];
        normals_tagged(seed, gid, lo, TAG_MH, hi, D, z);
        for (int d = 0; d < D; ++d) y[d] = fma(mc->v0[d], z[d], c->x[d]);
      } else if (mc->kind == MCG_MIX_KD_INTERP) {
        const or_kd* t = p->kd;
        rng4(seed, gid, lo, CALL_KD_PICK, TAG_MH, hi, w);
        uint32_t pk = or_randint(w[0], w[1], (uint32_t)t->M);
        int64_t L = kd_find_leaf_idx(t, t->pts + (int64_t)pk * D);
        const double* blo = t->lbox + L * 2 * D;
        const double* bhi = blo + D;
        for (int d = 0; d < D; d += 2) {
          rng4(seed, gid, lo, (uint32_t)(d >> 1), TAG_MH, hi, w);
          y[d] = blo[d] + (bhi[d] - blo[d]) * or_u53(w[0], w[1]);
          if (d + 1 < D) y[d + 1] = blo[d + 1] + (bhi[d + 1] - blo[d + 1]) * or_u53(w[2], w[3]);
        }
      } else {
        for (int d = 0; d < D; d += 2) {
          rng4(seed, gid, lo, (uint32_t)(d >> 1), TAG_MH, hi, w);
          double u0 = or_u53(w[0], w[1]), u1 = or_u53(w[2], w[3]);
          for (int j = 0; j < 2 && d + j < D; ++j) {
            int e = d + j;
            double uu = j ? u1 : u0;
            if (mc->kind == MCG_MIX_SHIFT_UNIFORM)   /* x + random_between a b (mcmc_test.ml:15-16) */
              y[e] = c->x[e] + (mc->v0[e] + mc->width[e] * uu);
            else
              y[e] = wrap_uniform(mc->v0[e], mc->v1[e], mc->v2[e], c->x[e], uu);
          }
        }
      }
      if (p->mix_kd) lqy = p->kd->llogq[kd_find_leaf_idx(p->kd, y)];
      lf = mix_log_jp(p, c->x, y, lqy);   /* log_jump_prob start proposed */
      lb = mix_log_jp(p, y, c->x, c->lq); /* log_jump_prob proposed start */
      break;
    }
    default: return -1;
  }
  double lly = lik_eval(p, y);
  double lpy = prior_eval(p, y);
  double post_y = lly + lpy;
  double post_x = c->ll + c->lp;
  double ratio = ((post_y - post_x) + lb) - lf;
  uint32_t w[4];
  rng4(seed, gid, lo, CALL_ACCEPT, TAG_MH, hi, w);
  const double u = or_u53(w[0], w[1]);
  double lu = g_literal ? log(u) : or_log(u);
  const int acc = lu < ratio;
  if (pr) {
    memcpy(pr->y, y, sizeof(double) * (size_t)D);
    pr->lly = lly; pr->lpy = lpy; pr->ratio = ratio; pr->u = u; pr->acc = acc;
  }
  if (acc) {
    for (int d = 0; d < D; ++d) c->x[d] = y[d];
    c->ll = lly; c->lp = lpy; c->lq = lqy;
    return 1;
  }
  return 0;
}

/* Shadow of the reference's literal arithmetic along a canonical chain: N chains run nsteps
 * canonical MH steps (what the GPU does) from (x [D][N], ll, lp) at global step step0; at every
 * step the SAME proposal is also judged with the literal arithmetic (literal ll of the current
 * and proposed points, glibc log of the same uniform).  flips[c] counts the steps whose accept
 * decision differs; max_rel_ll = max over all proposals of |ll_literal - ll_canonical| /
 * max(|ll|, 1) (relative, but absolute where ll crosses 0: near a peak the O(1) terms cancel);
 * min_margin = the smallest |log u - ratio| seen (how close any decision came to a flip). */
int or_mh_literal_shadow(const or_model* m, uint64_t seed, int64_t N, uint64_t step0, int64_t nsteps,
                         const double* x, const double* ll, const double* lp, int64_t* flips,
                         double* max_rel_ll, double* min_margin) {
  prep_t p;
  if (prep_model(m, &p) != 0 || g_literal) return -1;
  const int D = p.D;
  if (!(p.lik == MCG_LIK_DIAG_GAUSS || p.lik == MCG_LIK_GAUSS_SHELL || p.lik == MCG_LIK_GAUSS_MIX) || D > 256) {
    prep_free(&p);
    return -1;
  }
  step_probe* pr = (step_probe*)malloc(sizeof(step_probe));
  double mrel = 0.0, mmar = INFINITY;
  for (int64_t i = 0; i < N; ++i) {
    chain_t c;
    for (int d = 0; d < D; ++d) c.x[d] = x[(int64_t)d * N + i];
    c.ll = ll[i]; c.lp = lp[i]; c.lq = 0.0;
    int64_t f = 0;
    for (int64_t t = 0; t < nsteps; ++t) {
      const double llx_lit = lik_literal(&p, c.x), lpx = c.lp;
      mh_step(&p, seed, (uint32_t)i, step0 + (uint64_t)t, &c, pr);
      const double lly_lit = lik_literal(&p, pr->y);
      if (isfinite(pr->lly)) {
        const double rel = fabs(lly_lit - pr->lly) / fmax(fabs(pr->lly), 1.0);
        if (rel > mrel) mrel = rel;
      }
      const double ratio_lit = (lly_lit + pr->lpy) - (llx_lit + lpx);
      const int acc_lit = log(pr->u) < ratio_lit;
      f += acc_lit != pr->acc;
      const double mar = fabs(or_log(pr->u) - pr->ratio);
      if (mar < mmar) mmar = mar;
    }
    flips[i] = f;
  }
  free(pr);
  prep_free(&p);
  if (max_rel_ll) *max_rel_ll = mrel;
  if (min_margin) *min_margin = mmar;
  return 0;
}

/* ======================================================================================
 * Batched mcmc_array (mcmc.ml:58-72) with records, bitmap and running accumulators
 * ====================================================================================== */
typedef struct {
  const prep_t* p; uint64_t seed; uint32_t chain_offset; int64_t N; uint64_t step0;
  double* x; double* ll; double* lp; uint64_t* nacc; const or_run_opts* o;
  double* rec_x; double* rec_ll; double* rec_lp; uint64_t* bits; or_accum* acc;
  int64_t i0, i1; int status;
} mh_job;

/* log-space harmonic-mean partial (m, s) = (max v, sum exp(v - max)) of v = -ll
   (evidence.ml:101-107 in log space); s == 0 marks an empty partial. */
static void hm_update(double* m, double* s, double v) {
  if (*s == 0.0) { *m = v; *s = 1.0; return; }
  double e = (v == *m) ? 1.0 : or_exp(-fabs(v - *m));
  if (v > *m) { *s = *s * e + 1.0; *m = v; } else { *s = *s + e; }
}

static void hm_comb(double* ma, double* sa, double mb, double sb) {
  if (sb == 0.0) return;
  if (*sa == 0.0) { *ma = mb; *sa = sb; return; }
  double mm = (*ma > mb) ? *ma : mb;
  *sa = *sa * or_exp(*ma - mm) + sb * or_exp(mb - mm);
  *ma = mm;
}

/* the 8 record classes of one chain in the canonical tree ((0,4),(2,6)),((1,5),(3,7)) */
static void hm_classes(const or_accum* acc, int64_t N, int64_t c, double* m, double* s) {
  double cm[8], cs[8];
  for (int k = 0; k < 8; ++k) { cm[k] = acc->hm_m[k * N + c]; cs[k] = acc->hm_s[k * N + c]; }
  for (int k = 0; k < 4; ++k) hm_comb(&cm[k], &cs[k], cm[k + 4], cs[k + 4]);
  hm_comb(&cm[0], &cs[0], cm[2], cs[2]);
  hm_comb(&cm[1], &cs[1], cm[3], cs[3]);
  hm_comb(&cm[0], &cs[0], cm[1], cs[1]);
  *m = cm[0]; *s = cs[0];
}

static void record_sample(mh_job* j, int64_t i, int64_t r, const chain_t* c) {
  const or_run_opts* o = j->o;
  int D = j->p->D;
  int64_t N = j->N;
  if (o->record_x && j->rec_x)
    for (int d = 0; d < D; ++d) j->rec_x[(r * D + d) * N + i] = c->x[d];
  if (o->record_llp) {
    if (j->rec_ll) j->rec_ll[r * N + i] = c->ll;
    if (j->rec_lp) j->rec_lp[r * N + i] = c->lp;
  }
  if (o->accumulate && j->acc) {
    or_accum* a = j->acc;
    double inv = 1.0 / (double)(r + 1);
    for (int d = 0; d < D; ++d) {
      double* mean = &a->mean[(int64_t)d * N + i];
      double* m2 = &a->m2[(int64_t)d * N + i];
      double delta = c->x[d] - *mean;
      *mean = fma(delta, inv, *mean);
      *m2 = fma(delta, c->x[d] - *mean, *m2);
    }
    /* harmonic-mean partials in 8 record classes: record r updates class r & 7 */
    int64_t hc = (int64_t)(r & 7) * N + i;
    hm_update(&a->hm_m[hc], &a->hm_s[hc], -c->ll);
  }
}

static void* mh_worker(void* arg) {
  mh_job* j = (mh_job*)arg;
  const prep_t* p = j->p;
  const or_run_opts* o = j->o;
  int D = p->D;
  int64_t nsteps = o->nbin + (o->n_rec > 0 ? (o->n_rec - 1) * o->nskip : 0);
  int64_t words = (j->N + 63) / 64;
  chain_t c;
  for (int64_t i = j->i0; i < j->i1; ++i) {
    for (int d = 0; d < D; ++d) c.x[d] = j->x[(int64_t)d * j->N + i];
    c.ll = j->ll[i]; c.lp = j->lp[i];
    c.lq = 0.0;
    if (p->prop == MCG_PROP_KD_INTERP || p->mix_kd) c.lq = p->kd->llogq[kd_find_leaf_idx(p->kd, c.x)];
    uint32_t gid = j->chain_offset + (uint32_t)i;
    if (o->nbin == 0 && o->n_rec > 0) record_sample(j, i, 0, &c);
    uint64_t na = 0;
    for (int64_t t = 0; t < nsteps; ++t) {
      int a = mh_step(p, j->seed, gid, j->step0 + (uint64_t)t, &c, NULL);
      if (a < 0) { j->status = -1; return NULL; }
      na += (uint64_t)a;
      if (o->record_accept && j->bits && a)
        j->bits[t * words + (i >> 6)] |= (1ull << (i & 63));
      int64_t t1 = t + 1;
      if (t1 >= o->nbin && ((t1 - o->nbin) % o->nskip) == 0) {
        int64_t r = (t1 - o->nbin) / o->nskip;
        if (r < o->n_rec) record_sample(j, i, r, &c);
      }
    }
    for (int d = 0; d < D; ++d) j->x[(int64_t)d * j->N + i] = c.x[d];
    j->ll[i] = c.ll; j->lp[i] = c.lp;
    j->nacc[i] += na;
  }
  return NULL;
}

int or_mh_run(const or_model* m, uint64_t seed, uint32_t chain_offset, int64_t N, uint64_t step0,
              double* x, double* ll, double* lp, uint64_t* nacc, const or_run_opts* o,
              double* rec_x, double* rec_ll, double* rec_lp, uint64_t* accept_bits,
              or_accum* acc, int nthreads) {
  if (m->ndim < 1 || m->ndim > 256 || N < 1 || o->nskip < 1) return -1;
  prep_t p;
  if (prep_model(m, &p) != 0) return -1;
  if (nthreads < 1) nthreads = 1;
  int64_t blocks = (N + 63) / 64;
  if (nthreads > blocks) nthreads = (int)blocks;
  mh_job* jobs = (mh_job*)calloc((size_t)nthreads, sizeof(mh_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  int64_t per = (blocks + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    mh_job* j = &jobs[t];
    j->p = &p; j->seed = seed; j->chain_offset = chain_offset; j->N = N; j->step0 = step0;
    j->x = x; j->ll = ll; j->lp = lp; j->nacc = nacc; j->o = o;
    j->rec_x = rec_x; j->rec_ll = rec_ll; j->rec_lp = rec_lp; j->bits = accept_bits; j->acc = acc;
    j->i0 = t * per * 64; j->i1 = (t + 1) * per * 64;
    if (j->i0 > N) j->i0 = N;
    if (j->i1 > N) j->i1 = N;
  }
  if (nthreads == 1) mh_worker(&jobs[0]);
  else {
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, mh_worker, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  }
  int status = 0;
  for (int t = 0; t < nthreads; ++t) if (jobs[t].status) status = jobs[t].status;
  free(jobs); free(th);
  prep_free(&p);
  return status;
}

/* ======================================================================================
 * Reversible jump between two models (Mcmc.make_rjmcmc_sampler, mcmc.ml:89-119; rjmcmc_array's
 * schedule mcmc.ml:121-139), RNG injected: selector call CALL_RJ, start coin CALL_RJ_START
 * ====================================================================================== */
#define CALL_RJ 0xFFFF0006u
#define CALL_RJ_START 0xFFFF0007u

typedef struct {
  prep_t p[2];
  const or_rj_model* m[2];
  double logp[2];
  int DM;
} rj_prep;

/* log_jump_prob _ to of an independence jump; 0 for the random walks */
static double rj_ljp_to(const rj_prep* R, int k, int kind, const double* q, const double* to) {
  int D = R->m[k]->ndim;
  if (kind == MCG_RJ_JUMP_INDEP_GAUSS) {
    /* sum_d Stats.log_gaussian mu_d s_d to_d as C - S/2, e = to/s - mu/s (stats.ml:98-101) */
    double C = 0.0, S = 0.0;
    for (int d = 0; d < D; ++d) {
      double inv = 1.0 / q[D + d];
      double e = fma(to[d], inv, -(q[d] * inv));
      S = fma(e, e, S);
      C = C + (NEG_HALF_LOG_2PI - log(q[D + d]));
    }
    return C - 0.5 * S;
  } else if (kind == MCG_RJ_JUMP_KD) {
    const or_kd* t = (const or_kd*)R->m[k]->kd;
    return t->llogq[kd_find_leaf_idx(t, to)];
  }
  return 0.0;
}

static void rj_draw(const rj_prep* R, int k, int kind, const double* q, uint64_t seed, uint32_t gid,
                    uint32_t lo, uint32_t hi, const double* x, double* y) {
  int D = R->m[k]->ndim;
  for (int d = 0; d < R->DM; ++d) y[d] = 0.0;
  uint32_t w[4];
  if (kind == MCG_RJ_JUMP_GAUSS || kind == MCG_RJ_JUMP_INDEP_GAUSS) {
    double z[256];
    normals_tagged(seed, gid, lo, TAG_MH, hi, D, z);
    for (int d = 0; d < D; ++d) {
      double s = (kind == MCG_RJ_JUMP_GAUSS) ? (R->m[k]->n_jump == 1 ? q[0] : q[d]) : q[D + d];
      y[d] = (kind == MCG_RJ_JUMP_GAUSS) ? fma(s, z[d], x[d]) : fma(s, z[d], q[d]);
    }
  } else if (kind == MCG_RJ_JUMP_WRAP) {
    for (int d = 0; d < D; d += 2) {
      rng4(seed, gid, lo, (uint32_t)(d >> 1), TAG_MH, hi, w);
      y[d] = wrap_uniform(q[d], q[D + d], q[2 * D + d], x[d], or_u53(w[0], w[1]));
      if (d + 1 < D) y[d + 1] = wrap_uniform(q[d + 1], q[D + d + 1], q[2 * D + d + 1], x[d + 1], or_u53(w[2], w[3]));
    }
  } else {
    /* Interpolate_pdf.draw (interpolate_pdf.ml:114-119) on model k's tree */
    const or_kd* t = (const or_kd*)R->m[k]->kd;
    rng4(seed, gid, lo, CALL_KD_PICK, TAG_MH, hi, w);
    uint32_t pk = or_randint(w[0], w[1], (uint32_t)t->M);
    int64_t L = kd_find_leaf_idx(t, t->pts + (int64_t)pk * D);
    const double* blo = t->lbox + L * 2 * D;
    const double* bhi = blo + D;
    for (int d = 0; d < D; d += 2) {
      rng4(seed, gid, lo, (uint32_t)(d >> 1), TAG_MH, hi, w);
      y[d] = blo[d] + (bhi[d] - blo[d]) * or_u53(w[0], w[1]);
      if (d + 1 < D) y[d + 1] = blo[d + 1] + (bhi[d + 1] - blo[d + 1]) * or_u53(w[2], w[3]);
    }
  }
}

typedef struct {
  const rj_prep* R; uint64_t seed; int64_t N; const or_run_opts* o;
  uint8_t* tag; double* x; double* ll; double* lp; int draw_tags; const double* xa; const double* xb;
  double* rec_x; double* rec_ll; double* rec_lp; uint8_t* rec_tag; uint64_t* bits;
  uint64_t* nacc; uint64_t* nb_rec; int64_t i0, i1;
} rj_job;

static void* rj_worker(void* arg) {
  rj_job* j = (rj_job*)arg;
  const rj_prep* R = j->R;
  const or_run_opts* o = j->o;
  int DM = R->DM;
  int64_t N = j->N;
  int64_t nsteps = o->nbin + (o->n_rec > 0 ? (o->n_rec - 1) * o->nskip : 0);
  int64_t words = (N + 63) / 64;
  double x[256], y[256];
  for (int64_t i = j->i0; i < j->i1; ++i) {
    uint32_t gid = (uint32_t)i;
    int tag = j->tag[i];
    if (j->draw_tags) {              /* rjmcmc_array: is_a = Random.float 1.0 < 0.5 (mcmc.ml:123) */
      uint32_t w[4];
      rng4(j->seed, gid, 0u, CALL_RJ_START, TAG_MH, 0u, w);
      tag = or_u53(w[0], w[1]) < 0.5 ? 0 : 1;
    }
    int D0 = R->m[tag]->ndim;
    const double* src = tag ? j->xb : j->xa;
    for (int d = 0; d < DM; ++d) x[d] = d < D0 ? src[(int64_t)d * N + i] : 0.0;
    /* start record: log_like and lpa a + log pa (mcmc.ml:126-128) */
    double ll = lik_eval(&R->p[tag], x), lp = prior_eval(&R->p[tag], x) + R->logp[tag];
    uint64_t na = 0, nb = 0;
#define RJ_RECORD(r) do { \
      if (o->record_x && j->rec_x) for (int d = 0; d < DM; ++d) j->rec_x[((r) * DM + d) * N + i] = x[d]; \
      if (o->record_llp) { j->rec_ll[(r) * N + i] = ll; j->rec_lp[(r) * N + i] = lp; j->rec_tag[(r) * N + i] = (uint8_t)tag; } \
      nb += (uint64_t)tag; } while (0)
    if (o->nbin == 0 && o->n_rec > 0) RJ_RECORD(0);
    for (int64_t t = 0; t < nsteps; ++t) {
      uint64_t T = (uint64_t)t;
      uint32_t lo = (uint32_t)T, hi = (uint32_t)(T >> 32);
      uint32_t w[4];
      rng4(j->seed, gid, lo, CALL_RJ, TAG_MH, hi, w);
      const or_rj_model* mc = R->m[tag];
      int internal = or_u53(w[0], w[1]) < mc->model_prior;          /* mcmc.ml:94,99 */
      int ytag = internal ? tag : 1 - tag;
      const or_rj_model* my = R->m[ytag];
      int kind = internal ? my->jump_kind : my->into_kind;
      const double* q = internal ? my->jump_params : my->into_params;
      rj_draw(R, ytag, kind, q, j->seed, gid, lo, hi, x, y);
      double lf = R->logp[ytag] + rj_ljp_to(R, ytag, kind, q, y);  /* log_jump_prob x y */
      double lb = internal ? R->logp[ytag] + rj_ljp_to(R, ytag, kind, q, x)
                           : R->logp[tag] + rj_ljp_to(R, tag, mc->into_kind, mc->into_params, x);
      double lly = lik_eval(&R->p[ytag], y);
      double lpy = R->logp[ytag] + prior_eval(&R->p[ytag], y);
      double ratio = (((lly + lpy) - (ll + lp)) + lb) - lf;
      rng4(j->seed, gid, lo, CALL_ACCEPT, TAG_MH, hi, w);
      int a = or_log(or_u53(w[0], w[1])) < ratio;
      if (a) {
        for (int d = 0; d < DM; ++d) x[d] = y[d];
        ll = lly; lp = lpy; tag = ytag; ++na;
        if (o->record_accept && j->bits) j->bits[t * words + (i >> 6)] |= (1ull << (i & 63));
      }
      int64_t t1 = t + 1;
      if (t1 >= o->nbin && ((t1 - o->nbin) % o->nskip) == 0) {
        int64_t r = (t1 - o->nbin) / o->nskip;
        if (r < o->n_rec) RJ_RECORD(r);
      }
    }
#undef RJ_RECORD
    for (int d = 0; d < DM; ++d) j->x[(int64_t)d * N + i] = x[d];
    j->ll[i] = ll; j->lp[i] = lp; j->tag[i] = (uint8_t)tag;
    j->nacc[i] += na;
    if (o->accumulate) j->nb_rec[i] += nb;
  }
  return NULL;
}

int or_rj_run(const or_rj_model* a, const or_rj_model* b, uint64_t seed, int64_t N, uint8_t* tag,
              int draw_tags, const double* xa, const double* xb, double* x, double* ll, double* lp, uint64_t* nacc, uint64_t* nb_rec,
              const or_run_opts* o, double* rec_x, double* rec_ll, double* rec_lp, uint8_t* rec_tag,
              uint64_t* accept_bits, int nthreads) {
  rj_prep R;
  memset(&R, 0, sizeof R);
  R.m[0] = a; R.m[1] = b;
  R.DM = a->ndim > b->ndim ? a->ndim : b->ndim;
  if (a->ndim < 1 || b->ndim < 1 || R.DM > 256 || N < 1 || o->nskip < 1) return -1;
  double one = 1.0;
  for (int k = 0; k < 2; ++k) {
    const or_rj_model* q = R.m[k];
    or_model m = {q->ndim, q->lik_kind, q->lik_params, q->n_lik, q->prior_kind, q->prior_params,
                  q->n_prior, MCG_PROP_GAUSS, &one, 1, NULL};
    if (prep_model(&m, &R.p[k]) != 0) return -1;
    R.logp[k] = log(q->model_prior);
  }
  if (nthreads < 1) nthreads = 1;
  if (nthreads > N) nthreads = (int)N;
  rj_job* jobs = (rj_job*)calloc((size_t)nthreads, sizeof(rj_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  int64_t per = (N + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    rj_job* j = &jobs[t];
    j->R = &R; j->seed = seed; j->N = N; j->o = o; j->tag = tag; j->x = x; j->ll = ll; j->lp = lp;
    j->draw_tags = draw_tags; j->xa = xa; j->xb = xb; j->rec_x = rec_x; j->rec_ll = rec_ll; j->rec_lp = rec_lp;
    j->rec_tag = rec_tag; j->bits = accept_bits; j->nacc = nacc; j->nb_rec = nb_rec;
    j->i0 = t * per; j->i1 = (t + 1) * per;
    if (j->i0 > N) j->i0 = N;
    if (j->i1 > N) j->i1 = N;
  }
  /* accept bits of one 64-chain word must come from one thread: split on 64-chain blocks */
  if (nthreads > 1) {
    int64_t blocks = (N + 63) / 64, bper = (blocks + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; ++t) {
      jobs[t].i0 = t * bper * 64; jobs[t].i1 = (t + 1) * bper * 64;
      if (jobs[t].i0 > N) jobs[t].i0 = N;
      if (jobs[t].i1 > N) jobs[t].i1 = N;
    }
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, rj_worker, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  } else {
    rj_worker(&jobs[0]);
  }
  free(jobs); free(th);
  prep_free(&R.p[0]); prep_free(&R.p[1]);
  return 0;
}

/* ======================================================================================
 * Tile statistics: Chan/Welford pairwise combine + log-space harmonic-mean partials
 * ====================================================================================== */
static void comb(int D, double* a, const double* b) {
  /* entry layout: n, mean[D], m2[D], hm_m, hm_s */
  double na = a[0], nb = b[0];
  if (nb == 0.0) return;
  if (na == 0.0) { memcpy(a, b, sizeof(double) * (size_t)(2 * D + 3)); return; }
  double n = na + nb;
  double fb = nb / n;
  double fab = (na * nb) / n;
  for (int d = 0; d < D; ++d) {
    double delta = b[1 + d] - a[1 + d];
    a[1 + d] = a[1 + d] + delta * fb;
    a[1 + D + d] = (a[1 + D + d] + b[1 + D + d]) + (delta * delta) * fab;
  }
  double ma = a[2 * D + 1], sa = a[2 * D + 2], mb = b[2 * D + 1], sb = b[2 * D + 2];
  double mm = (ma > mb) ? ma : mb;
  a[2 * D + 1] = mm;
  a[2 * D + 2] = sa * or_exp(ma - mm) + sb * or_exp(mb - mm);
  a[0] = n;
}

void or_tile_stats(int D, int64_t N, int64_t nrec, const or_accum* acc, double* tiles) {
  int W = 2 * D + 3;
  int64_t ntiles = (N + 255) / 256;
  double* e = (double*)malloc(sizeof(double) * 256 * (size_t)W);
  for (int64_t t = 0; t < ntiles; ++t) {
    for (int i = 0; i < 256; ++i) {
      int64_t c = t * 256 + i;
      double* ei = e + (size_t)i * W;
      if (c < N && nrec > 0) {
        ei[0] = (double)nrec;
        for (int d = 0; d < D; ++d) {
          ei[1 + d] = acc->mean[(int64_t)d * N + c];
          ei[1 + D + d] = acc->m2[(int64_t)d * N + c];
        }
        hm_classes(acc, N, c, &ei[2 * D + 1], &ei[2 * D + 2]);
      } else {
        memset(ei, 0, sizeof(double) * (size_t)W);
        ei[2 * D + 1] = -INFINITY;
      }
    }
    for (int s = 128; s >= 1; s >>= 1)
      for (int i = 0; i < s; ++i) comb(D, e + (size_t)i * W, e + (size_t)(i + s) * W);
    memcpy(tiles + (size_t)t * W, e, sizeof(double) * (size_t)W);
  }
  free(e);
}

void or_combine_tiles(int D, int64_t ntiles, const double* tiles, double* mean, double* sd,
                      double* log_z_hm) {
  int W = 2 * D + 3;
  double* a = (double*)calloc((size_t)W, sizeof(double));
  a[2 * D + 1] = -INFINITY;
  for (int64_t t = 0; t < ntiles; ++t) comb(D, a, tiles + (size_t)t * W);
  double n = a[0];
  for (int d = 0; d < D; ++d) {
    mean[d] = a[1 + d];
    sd[d] = sqrt(a[1 + D + d] / (n - 1.0));
  }
  *log_z_hm = log(n) - (a[2 * D + 1] + log(a[2 * D + 2]));
  free(a);
}

double or_harmonic_mean_naive(const double* ll, int64_t n) {   /* evidence.ml:101-107 */
  double linv = 0.0;
  for (int64_t i = 0; i < n; ++i) linv = linv + 1.0 / exp(ll[i]);
  return (double)n / linv;
}

/* ======================================================================================
 * Nested sampling (nested.ml), slot semantics, k retired per generation
 * ====================================================================================== */
typedef struct { double ll; int64_t tie; int32_t slot; } nkey_t;

static int key_less(const nkey_t* a, const nkey_t* b) {
  if (a->ll < b->ll) return 1;
  if (a->ll > b->ll) return 0;
  return a->tie < b->tie;
}

static int key_cmp(const void* a, const void* b) {
  const nkey_t* x = (const nkey_t*)a;
  const nkey_t* y = (const nkey_t*)b;
  if (key_less(x, y)) return -1;
  if (key_less(y, x)) return 1;
  return 0;
}

/* log-sum of one generation's k > 1 terms v[0..n) (the k-at-a-time generalisation of the running
   estimate, nested.ml:138-141; k = 1 is the reference's plain fold): M = max v, then
   M + log(sum_i exp(v_i - M)) with the exps summed by a fixed pairwise tree (pad to a power of
   two with 0, add i + s into i).  The kernel (estimate_body, mcg_nested_kernels.hip) does the
   same operations in the same order. */
static double tree_lse(double* v, int64_t n) {
  double M = -INFINITY;
  for (int64_t i = 0; i < n; ++i) M = v[i] > M ? v[i] : M;
  if (M == -INFINITY) return -INFINITY;
  int64_t p2 = 1;
  while (p2 < n) p2 <<= 1;
  for (int64_t i = 0; i < n; ++i) v[i] = or_exp(v[i] - M);
  for (int64_t i = n; i < p2; ++i) v[i] = 0.0;
  for (int64_t s = p2 >> 1; s >= 1; s >>= 1)
    for (int64_t i = 0; i < s; ++i) v[i] = v[i] + v[i + s];
  return M + or_log(v[0]);
}

int or_nested(const or_model* m, uint64_t seed, const or_nested_opts* o, double* pts, double* lls,
              double* lps, double* log_wts, int64_t cap, or_nested_result* res) {
  prep_t p;
  if (prep_model(m, &p) != 0) return -1;
  int D = p.D;
  int64_t n = o->nlive, k = o->k;
  if (n < 2 || k < 1 || k >= n || D > 256 ||
      !(p.prior == MCG_PRIOR_BOX || p.prior == MCG_PRIOR_OPEN_BOX || p.prior == MCG_PRIOR_DIAG_GAUSS)) {
    prep_free(&p); return -1;
  }
  double* lx = (double*)malloc(sizeof(double) * (size_t)(n * D));   /* live AoS [slot][D] */
  double* lll = (double*)malloc(sizeof(double) * (size_t)n);
  double* llp = (double*)malloc(sizeof(double) * (size_t)n);
  nkey_t* keys = (nkey_t*)malloc(sizeof(nkey_t) * (size_t)n);
  nkey_t* nk = (nkey_t*)malloc(sizeof(nkey_t) * (size_t)n);
  double* nx = (double*)malloc(sizeof(double) * (size_t)(k * D));
  double* nll = (double*)malloc(sizeof(double) * (size_t)k);
  double* nlp = (double*)malloc(sizeof(double) * (size_t)k);
  int64_t p2 = 1; while (p2 < k) p2 <<= 1;
  double* tv = (double*)malloc(sizeof(double) * (size_t)p2);
  double* prefix = (double*)malloc(sizeof(double) * (size_t)(k + 1));
  /* prefix[j] = sum_{j'<j} log1p(-1/(n-j')) -- volume after j retirements in a generation */
  prefix[0] = 0.0;
  for (int64_t j = 0; j < k; ++j) prefix[j + 1] = prefix[j] + log1p(-1.0 / (double)(n - j));
  /* draw_prior: uniform in the box (Stats.draw_uniform, stats.ml:126-128), or for a DIAG_GAUSS
     prior Stats.draw_gaussian mu sigma per dim (stats.ml:113-124: mu + sigma z) with the normals
     of dims 4c .. 4c+3 from call c */
  for (int64_t s = 0; s < n; ++s) {
    if (p.prior == MCG_PRIOR_DIAG_GAUSS) {
      for (int c = 0; 4 * c < D; ++c) {
        uint32_t w[4];
        rng4(seed, (uint32_t)s, 0u, (uint32_t)c, TAG_NEST_PRIOR, 0u, w);
        for (int j = 0; j < 4 && 4 * c + j < D; ++j)
          lx[s * D + 4 * c + j] = p.gp_mu[4 * c + j] + p.gp_sig[4 * c + j] * or_normal(w[j]);
      }
    } else
    for (int d = 0; d < D; d += 2) {
      uint32_t w[4];
      rng4(seed, (uint32_t)s, 0u, (uint32_t)(d >> 1), TAG_NEST_PRIOR, 0u, w);
      lx[s * D + d] = p.lo[d] + (p.hi[d] - p.lo[d]) * or_u53(w[0], w[1]);
      if (d + 1 < D) lx[s * D + d + 1] = p.lo[d + 1] + (p.hi[d + 1] - p.lo[d + 1]) * or_u53(w[2], w[3]);
    }
    lll[s] = lik_eval(&p, lx + s * D);
    llp[s] = prior_eval(&p, lx + s * D);
    keys[s].ll = lll[s]; keys[s].tie = s; keys[s].slot = (int32_t)s;
  }
  qsort(keys, (size_t)n, sizeof(nkey_t), key_cmp);   /* total order: (ll, tie) unique */
  double sigma_de = 2.38 / sqrt(2.0 * (double)D);   /* mcmc.ml:212 */
  double log_vol = 0.0, est = -INFINITY;
  int64_t mrep = 0, ndead = 0, gen = 0;
  int status = 0;
  int64_t max_iter = o->max_iter > 0 ? o->max_iter : 1000 * n;
  for (;;) {
    double thr = keys[k - 1].ll;
    /* k constrained DE-MCMC walkers (nested.ml:50-74) */
    for (int64_t w = 0; w < k; ++w) {
      uint32_t wid = (uint32_t)(mrep + w);
      uint32_t rw[4];
      int64_t start = -1;
      for (uint32_t a = 0; a < 4096; ++a) {
        rng4(seed, wid, a, CALL_START, TAG_NEST_WALK, 0u, rw);
        uint32_t r = or_randint(rw[0], rw[1], (uint32_t)n);
        if (lll[r] >= thr) { start = r; break; }
      }
      if (start < 0) start = keys[k - 1].slot;
      double cur[256], y[256];
      for (int d = 0; d < D; ++d) cur[d] = lx[start * D + d];
      double cur_l = (lll[start] >= thr) ? llp[start] : -INFINITY;   /* mcmc_logl, :54-59 */
      for (int64_t s = 0; s < o->nmcmc; ++s) {
        rng4(seed, wid, (uint32_t)s, CALL_DE_IDX, TAG_NEST_WALK, 0u, rw);
        uint32_t i = or_randint(rw[0], rw[1], (uint32_t)n);
        uint32_t jj = or_randint(rw[2], rw[3], (uint32_t)(n - 1));
        uint32_t j = jj + (jj >= i);
        rng4(seed, wid, (uint32_t)s, CALL_DE_SCALE, TAG_NEST_WALK, 0u, rw);
        double dsc;
        if (o->mode_hop != 0.0 && or_u53(rw[0], rw[1]) < o->mode_hop) dsc = 1.0;
        else dsc = sigma_de * or_normal(rw[2]);
        for (int d = 0; d < D; ++d) y[d] = cur[d] + dsc * (lx[(int64_t)j * D + d] - lx[(int64_t)i * D + d]);
        double lly = lik_eval(&p, y);
        double ml = (lly >= thr) ? prior_eval(&p, y) : -INFINITY;
        double ratio = (((ml + 0.0) - (cur_l + 0.0)) + 0.0) - 0.0;
        rng4(seed, wid, (uint32_t)s, CALL_ACCEPT, TAG_NEST_WALK, 0u, rw);
        double uw = or_u53(rw[0], rw[1]);
        double lu = g_literal ? log(uw) : or_log(uw);
        if (lu < ratio) { for (int d = 0; d < D; ++d) cur[d] = y[d]; cur_l = ml; }
      }
      for (int d = 0; d < D; ++d) nx[w * D + d] = cur[d];
      nll[w] = lik_eval(&p, cur);
      nlp[w] = prior_eval(&p, cur);
      if (!(nll[w] >= thr)) status = -2;                    /* nested.ml:70-72 */
    }
    if (status) break;
    /* retire the k lowest (in key order), update the running estimate (nested.ml:138-141) */
    for (int64_t j = 0; j < k; ++j) {
      int32_t sl = keys[j].slot;
      if (ndead >= cap) { status = -1; break; }
      memcpy(pts + ndead * D, lx + (int64_t)sl * D, sizeof(double) * (size_t)D);
      lls[ndead] = lll[sl]; lps[ndead] = llp[sl];
      ++ndead;
      double nj = (double)(n - j);
      double lv = log_vol + prefix[j];
      double log_dv = o->ref_stop_quirk ? lv + 1.0 / nj : lv + log(1.0 / nj);
      tv[j] = lll[sl] + log_dv;
    }
    if (status) break;
    if (g_literal) {                     /* log_sum_logs per retired point (nested.ml:138-141) */
      for (int64_t j = 0; j < k; ++j) est = or_log_sum_logs(est, tv[j]);
    } else {
      est = (k == 1) ? or_plse(est, tv[0]) : or_plse(est, tree_lse(tv, k));
    }
    log_vol = log_vol + prefix[k];
    /* replace the retired slots (slot semantics of nested.ml:26-43) */
    for (int64_t j = 0; j < k; ++j) {
      int32_t sl = keys[j].slot;
      memcpy(lx + (int64_t)sl * D, nx + j * D, sizeof(double) * (size_t)D);
      lll[sl] = nll[j]; llp[sl] = nlp[j];
      nk[j].ll = nll[j]; nk[j].tie = -(mrep + j + 1); nk[j].slot = sl;
    }
    qsort(nk, (size_t)k, sizeof(nkey_t), key_cmp);
    /* merge survivors keys[k..n) with new sorted nk[0..k) */
    {
      nkey_t* out = (nkey_t*)malloc(sizeof(nkey_t) * (size_t)n);
      int64_t a = k, b = 0, q = 0;
      while (a < n && b < k) out[q++] = key_less(&nk[b], &keys[a]) ? nk[b++] : keys[a++];
      while (a < n) out[q++] = keys[a++];
      while (b < k) out[q++] = nk[b++];
      memcpy(keys, out, sizeof(nkey_t) * (size_t)n);
      free(out);
    }
    mrep += k; ++gen;
    /* remaining_integral_negligable (nested.ml:45-48) on the replaced live set */
    double live_est = log_vol + keys[n - 1].ll;
    const double tot = g_literal ? or_log_sum_logs(est, live_est) : or_plse(est, live_est);
    if (live_est - tot <= log(o->epsrel)) break;
    if (ndead >= max_iter) break;
  }
  int64_t ntot = ndead + n;
  if (status == 0 && ntot > cap) status = -1;
  if (status == 0) {
    for (int64_t j = 0; j < n; ++j) {
      int32_t sl = keys[j].slot;
      memcpy(pts + (ndead + j) * D, lx + (int64_t)sl * D, sizeof(double) * (size_t)D);
      lls[ndead + j] = lll[sl]; lps[ndead + j] = llp[sl];
    }
    or_evidence_weights(ntot, n, k, lls, &res->log_ev, &res->log_dev, log_wts);
  }
  res->n_dead = ndead; res->n_total = ntot; res->n_gen = gen; res->status = status;
  free(lx); free(lll); free(llp); free(keys); free(nk); free(nx); free(nll); free(nlp);
  free(tv); free(prefix);
  prep_free(&p);
  return status;
}

/* nested.ml:81-120.  Dead point i was retired with n_i = nlive - (i mod k) live points; its
   remaining volume is logX_i = (i div k) * L_k + prefix[i mod k].  With k = 1 this is exactly
   log_vol_fraction + i * log_reduction_frac of nested.ml:96. */
#define OR_EV_BLOCK 65536
void or_evidence_weights(int64_t n, int64_t nlive, int64_t k, const double* ll,
                         double* log_ev, double* log_dev, double* wts) {
  const double log_half = -0.69314718055994530942;
  int64_t ilive = n - nlive;
  double* prefix = (double*)malloc(sizeof(double) * (size_t)(k + 1));
  prefix[0] = 0.0;
  for (int64_t j = 0; j < k; ++j) prefix[j + 1] = prefix[j] + log1p(-1.0 / (double)(nlive - j));
  for (int64_t i = 0; i < n; ++i) wts[i] = -INFINITY;
  /* the running sums low / high fold the iterations in blocks of OR_EV_BLOCK: a sequential
     log-sum inside each block from -inf, then a sequential log-sum of the block results -- the
     reference's sequential fold exactly when n <= OR_EV_BLOCK (a single block), and within
     rounding of it otherwise (the blocks run in parallel on the host) */
  double low = -INFINITY, high = -INFINITY, blow = -INFINITY, bhigh = -INFINITY;
  int64_t it = 0;
#define OR_EV_FOLD(dl_, dh_) do { \
    blow = or_log_sum_logs(blow, (dl_)); bhigh = or_log_sum_logs(bhigh, (dh_)); \
    if (++it % OR_EV_BLOCK == 0 || it == n) { \
      low = or_log_sum_logs(low, blow); high = or_log_sum_logs(high, bhigh); \
      blow = -INFINITY; bhigh = -INFINITY; } } while (0)
  for (int64_t i = 0; i < ilive; ++i) {
    int64_t j = i % k, g = i / k;
    double logx = (double)g * prefix[k] + prefix[j];
    double log_dv = log(1.0 / (double)(nlive - j)) + logx;
    if (k == 1) log_dv = log(1.0 / (double)nlive) + (double)i * log1p(-1.0 / (double)nlive);
    double dlow = log_dv + ll[i], dhigh = log_dv + ll[i + 1];
    OR_EV_FOLD(dlow, dhigh);
    wts[i] = or_log_sum_logs(wts[i], log_half + dlow);
    wts[i + 1] = or_log_sum_logs(wts[i + 1], log_half + dhigh);
  }
  /* the final live points each get 1/nlive of the volume that remained before the last
     retirement (nested.ml:104: log_vol_fraction + log X_(ilive-1)); for k > 1 that X is the
     generation prefix of the first ilive - 1 retirements (not the last dead point's own element,
     which divides by its live count nlive - k + 1); with no dead point at all, k = 1 keeps the
     reference's formula at i = -1 and k > 1 shares the whole prior volume */
  double log_dv;
  if (k == 1) log_dv = log(1.0 / (double)nlive) + (double)(ilive - 1) * log1p(-1.0 / (double)nlive);
  else if (ilive > 0) {
    int64_t m = ilive - 1, j = m % k, g = m / k;
    log_dv = log(1.0 / (double)nlive) + ((double)g * prefix[k] + prefix[j]);
  } else log_dv = log(1.0 / (double)nlive);
  for (int64_t i = ilive; i < n; ++i) {
    double dlow = log_dv + ll[i - 1], dhigh = log_dv + ll[i];
    OR_EV_FOLD(dlow, dhigh);
    wts[i - 1] = or_log_sum_logs(wts[i - 1], log_half + dlow);
    wts[i] = or_log_sum_logs(wts[i], log_half + dhigh);
  }
#undef OR_EV_FOLD
  *log_ev = log_half + or_log_sum_logs(low, high);
  *log_dev = high + log1p(-exp(low - high));
  for (int64_t i = 0; i < n; ++i) wts[i] = wts[i] - *log_ev;
  free(prefix);
}

double or_log_total_error_estimate(double log_ev, double log_dev, int64_t nlive) {
  double lre2 = -log((double)nlive);                                     /* nested.ml:148-150 */
  return 0.5 * or_log_sum_logs(2.0 * log_dev, lre2 + 2.0 * log_ev);
}

int64_t or_weight_binary_search_index(double x, const double* sums, int64_t n) { /* :152-165 */
  if (x <= sums[0]) return 0;
  int64_t lo = 0, hi = n - 1;
  while (hi - lo > 1) {
    int64_t mid = (lo + hi) / 2;
    if (x <= sums[mid]) hi = mid; else lo = mid;
  }
  return hi;
}

/* Nested.posterior_samples (nested.ml:167-178) as indices, RNG injected: summed weights
 * sequentially with glibc exp (:170-173), draw i of call `call` = u53 of Philox
 * (i lo, i hi, call, tag 5), then weight_binary_search_index (:152-165). */
void or_posterior_indices(uint64_t seed, uint32_t call, const double* log_wts, int64_t npts, int64_t n,
                          int64_t* idx) {
  double* sums = (double*)malloc((size_t)npts * sizeof(double));
  sums[0] = exp(log_wts[0]);
  for (int64_t i = 1; i < npts; ++i) sums[i] = exp(log_wts[i]) + sums[i - 1];
  for (int64_t i = 0; i < n; ++i) {
    uint32_t w[4];
    rng4(seed, (uint32_t)i, (uint32_t)((uint64_t)i >> 32), call, TAG_POSTERIOR, 0, w);
    idx[i] = or_weight_binary_search_index(or_u53(w[0], w[1]), sums, npts);
  }
  free(sums);
}

/* ======================================================================================
 * kD tree build (kd_tree.ml:155-175) -- geometry is deterministic: the i-th order statistic
 * found by the randomized find_ith (kd_tree.ml:69-86) is unique, so a sort replaces it.
 * ====================================================================================== */
typedef struct { const double* pts; int D; int dim; } sortctx_t;
static __thread sortctx_t g_sc;
static int cmp_idx_dim(const void* a, const void* b) {
  double x = g_sc.pts[(int64_t)(*(const int64_t*)a) * g_sc.D + g_sc.dim];
  double y = g_sc.pts[(int64_t)(*(const int64_t*)b) * g_sc.D + g_sc.dim];
  return (x < y) ? -1 : (x > y) ? 1 : 0;
}

static int32_t kd_new_node(or_kd* t) {
  if (t->nn == t->cap_n) {
    t->cap_n = t->cap_n ? 2 * t->cap_n : 64;
    t->dim = (int32_t*)realloc(t->dim, sizeof(int32_t) * (size_t)t->cap_n);
    t->split = (double*)realloc(t->split, sizeof(double) * (size_t)t->cap_n);
    t->right = (int32_t*)realloc(t->right, sizeof(int32_t) * (size_t)t->cap_n);
    t->leaf = (int32_t*)realloc(t->leaf, sizeof(int32_t) * (size_t)t->cap_n);
  }
  return (int32_t)t->nn++;
}

static int32_t kd_new_leaf(or_kd* t, int32_t count, const double* lo, const double* hi) {
  if (t->nl == t->cap_l) {
    t->cap_l = t->cap_l ? 2 * t->cap_l : 64;
    t->lcount = (int32_t*)realloc(t->lcount, sizeof(int32_t) * (size_t)t->cap_l);
    t->lbox = (double*)realloc(t->lbox, sizeof(double) * (size_t)t->cap_l * 2 * (size_t)t->D);
    t->llogq = (double*)realloc(t->llogq, sizeof(double) * (size_t)t->cap_l);
  }
  int32_t L = (int32_t)t->nl++;
  t->lcount[L] = count;
  memcpy(t->lbox + (int64_t)L * 2 * t->D, lo, sizeof(double) * (size_t)t->D);
  memcpy(t->lbox + (int64_t)L * 2 * t->D + t->D, hi, sizeof(double) * (size_t)t->D);
  /* jump_prob = nobjs / (v * n) (interpolate_pdf.ml:135-142), v = bounds_volume (kd_tree.ml:177-182) */
  double v = 1.0;
  for (int d = 0; d < t->D; ++d) v = v * (hi[d] - lo[d]);
  v = v + 0.0;
  t->llogq[L] = log((double)count / (v * (double)t->M));
  return L;
}

/* build over idx[0..n) with cell box lo/hi; preorder layout: left child = node + 1 */
static int32_t kd_build_rec(or_kd* t, const double* pts, int64_t* idx, int64_t n,
                            const double* lo, const double* hi) {
  int D = t->D;
  int32_t node = kd_new_node(t);
  int all_eq = 1;
  for (int64_t i = 1; i < n && all_eq; ++i)
    for (int d = 0; d < D; ++d)
      if (pts[idx[i] * D + d] != pts[idx[0] * D + d]) { all_eq = 0; break; }
  if (n == 1 || all_eq) {                                  /* kd_tree.ml:158-160 */
    t->dim[node] = -1; t->split[node] = 0.0; t->right[node] = -1;
    t->leaf[node] = kd_new_leaf(t, (int32_t)n, lo, hi);
    return node;
  }
  /* bounds_of_objects + longest_dim (kd_tree.ml:96-110, 120-130) */
  double* bl = (double*)malloc(sizeof(double) * D);
  double* bh = (double*)malloc(sizeof(double) * D);
  for (int d = 0; d < D; ++d) bl[d] = bh[d] = pts[idx[0] * D + d];
  for (int64_t i = 1; i < n; ++i)
    for (int d = 0; d < D; ++d) {
      double c = pts[idx[i] * D + d];
      if (c < bl[d]) bl[d] = c;
      if (c > bh[d]) bh[d] = c;
    }
  int dim = -1; double dxm = -INFINITY;
  for (int d = 0; d < D; ++d) { double dx = bh[d] - bl[d]; if (dx > dxm) { dim = d; dxm = dx; } }
  free(bl); free(bh);
  /* pivot = (n/2)-th order statistic along dim; lte = coord <= pivot (kd_tree.ml:162-168) */
  sortctx_t saved = g_sc;
  g_sc.pts = pts; g_sc.D = D; g_sc.dim = dim;
  qsort(idx, (size_t)n, sizeof(int64_t), cmp_idx_dim);
  g_sc = saved;
  double pv = pts[idx[n / 2] * D + dim];
  int64_t nlte = 0;
  while (nlte < n && pts[idx[nlte] * D + dim] <= pv) ++nlte;
  if (nlte == n) {                                         /* adjust_for_empty_split :150-152 */
    double mx = pts[idx[n - 1] * D + dim];
    nlte = 0;
    while (nlte < n && pts[idx[nlte] * D + dim] < mx) ++nlte;
  }
  double lt_bound = pts[idx[nlte - 1] * D + dim];          /* find_max comp lte */
  double gt_bound = pts[idx[nlte] * D + dim];              /* find_min comp gt */
  double x = 0.5 * (lt_bound + gt_bound);                  /* split_bounds :112-118 */
  double* nhi = (double*)malloc(sizeof(double) * D);
  double* nlo = (double*)malloc(sizeof(double) * D);
  memcpy(nhi, hi, sizeof(double) * D); nhi[dim] = x;
  memcpy(nlo, lo, sizeof(double) * D); nlo[dim] = x;
  t->dim[node] = dim; t->split[node] = x; t->leaf[node] = -1;
  kd_build_rec(t, pts, idx, nlte, lo, nhi);
  int32_t r = kd_build_rec(t, pts, idx + nlte, n - nlte, nlo, hi);
  t->right[node] = r;
  free(nhi); free(nlo);
  return node;
}

or_kd* or_kd_build(const double* pts, int64_t M, int D, const double* low, const double* high) {
  if (M < 1 || D < 1) return NULL;
  or_kd* t = (or_kd*)calloc(1, sizeof(or_kd));
  t->D = D; t->M = M;
  t->root_lo = (double*)malloc(sizeof(double) * D);
  t->root_hi = (double*)malloc(sizeof(double) * D);
  memcpy(t->root_lo, low, sizeof(double) * D);
  memcpy(t->root_hi, high, sizeof(double) * D);
  int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * (size_t)M);
  for (int64_t i = 0; i < M; ++i) idx[i] = i;
  kd_build_rec(t, pts, idx, M, low, high);
  free(idx);
  t->pts = (double*)malloc(sizeof(double) * (size_t)(M * D));
  memcpy(t->pts, pts, sizeof(double) * (size_t)(M * D));
  return t;
}

void or_kd_free(or_kd* t) {
  if (!t) return;
  free(t->pts);
  free(t->dim); free(t->split); free(t->right); free(t->leaf);
  free(t->lcount); free(t->lbox); free(t->llogq); free(t->root_lo); free(t->root_hi);
  free(t);
}

int64_t or_kd_nnodes(const or_kd* t) { return t->nn; }
int64_t or_kd_nleaves(const or_kd* t) { return t->nl; }

void or_kd_export(const or_kd* t, int32_t* node_dim, double* node_split, int32_t* node_right,
                  int32_t* node_leaf, int32_t* leaf_count, double* leaf_box) {
  memcpy(node_dim, t->dim, sizeof(int32_t) * (size_t)t->nn);
  memcpy(node_split, t->split, sizeof(double) * (size_t)t->nn);
  memcpy(node_right, t->right, sizeof(int32_t) * (size_t)t->nn);
  memcpy(node_leaf, t->leaf, sizeof(int32_t) * (size_t)t->nn);
  memcpy(leaf_count, t->lcount, sizeof(int32_t) * (size_t)t->nl);
  memcpy(leaf_box, t->lbox, sizeof(double) * (size_t)t->nl * 2 * (size_t)t->D);
}

/* find_cell (interpolate_pdf.ml:101-109): go left iff pt lies in the left child's (inclusive)
   box.  Boxes nest, so a point outside the root box always goes right; inside, the left test
   reduces to pt[dim] <= split. */
static int64_t kd_find_leaf_idx(const or_kd* t, const double* pt) {
  int inside = 1;
  for (int d = 0; d < t->D; ++d) inside &= (pt[d] >= t->root_lo[d]) & (pt[d] <= t->root_hi[d]);
  int32_t node = 0;
  while (t->dim[node] >= 0) {
    int left = inside && (pt[t->dim[node]] <= t->split[node]);
    node = left ? node + 1 : t->right[node];
  }
  return t->leaf[node];
}

int64_t or_kd_find_leaf(const or_kd* t, const double* pt) { return kd_find_leaf_idx(t, pt); }
double or_kd_log_jump_prob(const or_kd* t, const double* pt) { return t->llogq[kd_find_leaf_idx(t, pt)]; }
double or_kd_jump_prob(const or_kd* t, const double* pt) {
  int64_t L = kd_find_leaf_idx(t, pt);
  const double* lo = t->lbox + L * 2 * t->D;
  const double* hi = lo + t->D;
  double v = 1.0;
  for (int d = 0; d < t->D; ++d) v = v * (hi[d] - lo[d]);
  v = v + 0.0;
  return (double)t->lcount[L] / (v * (double)t->M);
}
