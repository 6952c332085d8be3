/*
 * oracle.h -- CPU restatement of farr/mcmc-ocaml's hot path (TEST INFRASTRUCTURE).
 *
 * This is the parity CHECKER, never the product.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product (libmcg.so) never links it.
 *
 * Parity status:
 *   - deterministic functions (Stats.* KATs, log_sum_logs, evidence_error_and_weights,
 *     kd-tree geometry) are pinned by the reference's own known-answer tests
 *     (test/stats_test.ml:5-55,94-120) and fixtures generated from this restatement;
 *   - RNG-driven paths (MH step, nested sampling) are pinned only STATISTICALLY against the
 *     reference's own tests (test/mcmc_test.ml, test/nested_test.ml, test/evidence_test.ml):
 *     the OCaml stdlib Random stream is irreproducible here (no OCaml toolchain, seeds come
 *     from /dev/random in test/run_tests.ml:14-18) -- bitwise parity vs OCaml is UNPINNED;
 *     bitwise parity GPU <-> this oracle is exact on the shared Philox stream.
 */
#ifndef MCG_ORACLE_H
#define MCG_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- RNG + portable math (spec in DESIGN.md §RNG) ---- */
void or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double or_u53(uint32_t w0, uint32_t w1);
uint32_t or_randint(uint32_t w0, uint32_t w1, uint32_t n);
double or_log(double x);
double or_exp(double x);
double or_sqrt(double x);
double or_normal(uint32_t w);
double or_plog1p(double r);
double or_plse(double a, double b);
/* normals for the MH proposal of chain c at step t: z[0..D) */
void or_step_normals(uint64_t seed, uint32_t chain, uint64_t step, uint32_t tag, int D, double* z);

/* Mcmc.uniform_wrapping (mcmc.ml:187-196) with the uniform u injected */
double or_wrap_uniform(double xmin, double xmax, double dx, double x, double u);

/* ---- Stats restatements (stats.ml) ---- */
double or_log_sum_logs(double a, double b);                      /* stats.ml:240-248 */
double or_mean(const double* xs, int64_t n);                     /* stats.ml:17-23 */
double or_std(const double* xs, int64_t n);                      /* stats.ml:35-43 */
void or_multi_mean(const double* xs, int64_t n, int d, double* mu);      /* stats.ml:58-70, xs [n][d] */
void or_multi_std(const double* xs, int64_t n, int d, double* sd);       /* stats.ml:72-87 */
double or_log_gaussian(double mu, double sigma, double x);      /* stats.ml:98-101 */
double or_log_cauchy(double x0, double gamma, double x);        /* stats.ml:93-96 */
double or_log_multi_gaussian(const double* mu, const double* sigma, const double* x, int d); /* :103-108 */
double or_log_lognormal(double mu, double sigma, double x);     /* stats.ml:217-221 */

/* ---- model descriptors (same parameter layouts as include/mcg.h) ---- */
typedef struct {
  int32_t ndim;
  int32_t lik_kind;            /* MCG_LIK_* */
  const double* lik_params;
  int64_t n_lik_params;
  int32_t prior_kind;          /* MCG_PRIOR_* */
  const double* prior_params;
  int64_t n_prior_params;
  int32_t prop_kind;           /* MCG_PROP_* */
  const double* prop_params;
  int64_t n_prop_params;
  /* KD_INTERP proposal: flattened tree (or_kd_build output) */
  const void* kd;
} or_model;

/* log-likelihood / log-prior of one point (x contiguous, length ndim) */
double or_loglik(const or_model* m, const double* x);
double or_logprior(const or_model* m, const double* x);

/* ---- batched MH (Mcmc.mcmc_array semantics per chain, mcmc.ml:58-72) ---- */
typedef struct {
  int64_t nbin, nskip, n_rec;
  int32_t record_x, record_llp, record_accept, accumulate;
} or_run_opts;

typedef struct {
  /* per-chain accumulators over recorded samples: mean/m2 [D][N] (Welford), hm_m/hm_s [8][N]
     log-space harmonic-mean partials of the 8 record classes r & 7 (s == 0: empty) */
  double* mean; double* m2; double* hm_m; double* hm_s;
} or_accum;

/* Runs nbin + (n_rec-1)*nskip steps on N chains, starting at global step `step0`.
   x [D][N] in/out, ll/lp [N] in/out, nacc [N] in/out (incremented).
   rec_x [n_rec][D][N], rec_ll/rec_lp [n_rec][N], accept_bits [nsteps][ceil(N/64)] u64.
   nthreads: chains are split into contiguous blocks, one per thread. */
/* ---- reversible jump between two models (Mcmc.make_rjmcmc_sampler, mcmc.ml:89-153) ----
   jump / into kinds and parameter layouts as MCG_RJ_JUMP_* in include/mcg.h; kd = or_kd tree */
typedef struct {
  int32_t ndim;
  int32_t lik_kind; const double* lik_params; int64_t n_lik;
  int32_t prior_kind; const double* prior_params; int64_t n_prior;
  int32_t jump_kind; const double* jump_params; int64_t n_jump;
  int32_t into_kind; const double* into_params; int64_t n_into;
  const void* kd;
  double model_prior;
} or_rj_model;
/* xa [D_A][N], xb [D_B][N] start points; x [Dmax][N] out (final states); tag [N] (in: start
   models unless draw_tags; out: final); rec_* [n_rec][..][N]; nb_rec [N] += recorded samples in
   model B when o->accumulate */
int or_rj_run(const or_rj_model* a, const or_rj_model* b, uint64_t seed, int64_t N, uint8_t* tag,
              int draw_tags, const double* xa, const double* xb, double* x, double* ll, double* lp, uint64_t* nacc, uint64_t* nb_rec,
              const or_run_opts* o, double* rec_x, double* rec_ll, double* rec_lp,
              uint8_t* rec_tag, uint64_t* accept_bits, int nthreads);

int or_mh_run(const or_model* m, uint64_t seed, uint32_t chain_offset, int64_t N, uint64_t step0,
              double* x, double* ll, double* lp, uint64_t* nacc, const or_run_opts* o,
              double* rec_x, double* rec_ll, double* rec_lp, uint64_t* accept_bits,
              or_accum* acc, int nthreads);

/* The reference's literal arithmetic instead of the GPU's canonical one (oracle.c):
   process-wide switch; or_mh_literal_shadow judges every canonical step's proposal both ways. */
void or_set_literal(int on);
int or_get_literal(void);
int or_mh_literal_shadow(const or_model* m, uint64_t seed, int64_t N, uint64_t step0, int64_t nsteps,
                         const double* x, const double* ll, const double* lp, int64_t* flips,
                         double* max_rel_ll, double* min_margin);

/* Tile reduction of the accumulators: 256-chain tiles, fixed pairwise tree.
   out per tile: [n, mean[D], m2[D], hm_m, hm_s] (2D+3 doubles). */
void or_tile_stats(int D, int64_t N, int64_t nrec, const or_accum* acc, double* tiles);
/* combine tiles in order -> mean[D], std[D], log Z_HM */
void or_combine_tiles(int D, int64_t ntiles, const double* tiles, double* mean, double* sd,
                      double* log_z_hm);

/* Evidence.evidence_harmonic_mean (evidence.ml:101-107), naive sequential */
double or_harmonic_mean_naive(const double* ll, int64_t n);

/* ---- nested sampling (nested.ml:122-178) ---- */
typedef struct {
  int64_t nlive, nmcmc, k;
  double epsrel, mode_hop;
  int32_t ref_stop_quirk;     /* nested.ml:140 quirk (default 1) */
  int64_t max_iter;           /* safety cap on dead points */
} or_nested_opts;

typedef struct {
  double log_ev, log_dev;
  int64_t n_dead, n_total, n_gen;
  int32_t status;             /* 0 ok, -2 Failure (constraint violated) */
} or_nested_result;

/* Returns all points (dead then live sorted) into pts [n_total][D], ll/lp [n_total],
   log_wts [n_total]; buffers sized cap (returns -1 if too small). */
int or_nested(const or_model* m, uint64_t seed, const or_nested_opts* o,
              double* pts, double* ll, double* lp, double* log_wts, int64_t cap,
              or_nested_result* res);

/* nested.ml:81-120, generalised to per-point live counts n_i (k=1 -> reference formula). */
void or_evidence_weights(int64_t n, int64_t nlive, int64_t k, const double* ll,
                         double* log_ev, double* log_dev, double* log_wts);
double or_log_total_error_estimate(double log_ev, double log_dev, int64_t nlive); /* :148-150 */
int64_t or_weight_binary_search_index(double x, const double* sums, int64_t n);  /* :152-165 */
void or_posterior_indices(uint64_t seed, uint32_t call, const double* log_wts, int64_t npts, int64_t n,
                          int64_t* idx);                                            /* :167-178 */

/* ---- kD tree / Interpolate_pdf (kd_tree.ml:155-175, interpolate_pdf.ml:80-142) ---- */
typedef struct or_kd or_kd;
or_kd* or_kd_build(const double* pts /*[M][D]*/, int64_t M, int D, const double* low, const double* high);
void or_kd_free(or_kd*);
int64_t or_kd_nnodes(const or_kd*);
int64_t or_kd_nleaves(const or_kd*);
/* flattened export: node_dim[nn] (-1 leaf), node_split[nn], node_right[nn], node_leaf[nn],
   leaf_count[nl], leaf_box[nl][2][D], root box low/high */
void or_kd_export(const or_kd*, int32_t* node_dim, double* node_split, int32_t* node_right,
                  int32_t* node_leaf, int32_t* leaf_count, double* leaf_box);
int64_t or_kd_find_leaf(const or_kd*, const double* pt);
double or_kd_log_jump_prob(const or_kd*, const double* pt);
double or_kd_jump_prob(const or_kd*, const double* pt);

#ifdef __cplusplus
}
#endif
#endif
