/*
 * mcg.h -- C-ABI of the MI355X-native batched sampler (libmcg.so).
 *
 * Drop-in boundary for farr/mcmc-ocaml's hot path.  Every entry point replaces a reference
 * interface (cited file:line, paths relative to the reference root); an OCaml host binds these
 * through ctypes / C stubs, the Python mirror in mcmc-ocaml_amd/mcmc_amd does the
 * same through ctypes.  Plain pointers and sizes only; no torch / HIP types cross this boundary.
 *
 * Conventions
 *   - Caller owns every host buffer; the context owns every device buffer.
 *   - Chain / point coordinates cross the boundary structure-of-arrays: x[d*N + i] ([D][N], C
 *     order) -- maps 1:1 to an OCaml Bigarray.Array2 c_layout or a numpy (D, N) array.
 *   - Return 0 on success, a negative MCG_E* code on error (the OCaml stub raises
 *     Invalid_argument for MCG_EINVAL, Failure for MCG_EFAIL, as the reference does at
 *     kd_tree.ml:70,97 / nested.ml:71).  mcg_last_error() gives the message.
 *   - No globals: the reference's global accept/reject counters (mcmc.ml:27-28) and global
 *     Random state become per-context state, so contexts are reentrant (one per host thread).
 *   - The reference's OCaml closures (log_likelihood, log_prior, jump_proposal, log_jump_prob;
 *     mcmc.mli:58-60) become data descriptors (kind + parameter vector) that a GPU kernel can run.
 */
#ifndef MCG_H
#define MCG_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCG_ABI_VERSION 3

/* ---- status codes ---- */
enum {
  MCG_OK = 0,
  MCG_EINVAL = -1,    /* Invalid_argument */
  MCG_EFAIL = -2,     /* Failure (e.g. nested.ml:70-72 constraint violation) */
  MCG_EDEVICE = -3,   /* HIP runtime error / no device / extension not loaded */
  MCG_ENOMEM = -4,
  MCG_ESTATE = -5     /* call out of order (e.g. mcg_run before mcg_init) */
};

/* ---- likelihood kinds (replace the log_likelihood closure, mcmc.mli:58) ----
   parameter layouts (doubles):
   DIAG_GAUSS    : mu[D], sigma[D]        Stats.log_multi_gaussian (stats.ml:103-108)
   FULLCOV_GAUSS : mu[D], U[D*D]          U = upper Cholesky factor of the precision, row major;
                                          ll = -D/2 log 2pi + sum log U_ii - 1/2 |U (x-mu)|^2
   GAUSS_SHELL   : c[D], r, w             ll = -log(sqrt(2 pi) w) - (|x-c| - r)^2 / (2 w^2)
   GAUSS_DATA    : nd, data[nsamp*nd]     D = 2 nd, x = (mu[nd], sigma[nd]); sum over data of
                                          Stats.log_gaussian (bin/gaussian_cauchy.ml:149-164)
   CAUCHY_DATA   : nd, data[nsamp*nd]     same with Stats.log_cauchy
   FLAT          : (none)                 ll = 0
   GAUSS_MIX     : m, then per component  ll = log (sum_i exp g_i), g_i = Stats.log_multi_gaussian
                   mu_i[D], sigma_i[D]    mu_i sigma_i x: the multimodal target of
                                          test/nested_test.ml:41-64 (1 <= m <= MCG_LIK_MIX_MAX);
                                          summed max-shifted, so where every g_i < ~-745 the
                                          result is finite while the reference's literal
                                          log (exp g1 + ...) underflows to -inf (its own test,
                                          D = 2, never gets there; the oracle's literal mode
                                          restates the reference's form)
   Any ndim >= 1 works for FLAT, DIAG_GAUSS, GAUSS_SHELL and GAUSS_MIX (FULLCOV_GAUSS: ndim <= 64):
   a dimension without compiled kernels runs on the next compiled width with zero-padded dims
   (zero likelihood terms, zero proposal steps, unbounded box); the padding never crosses this
   boundary.  The DATA kinds take nd <= 4.  The kD proposal runs at ndim 1-16 on every kind
   and 17-32 on FLAT, DIAG_GAUSS and GAUSS_SHELL (the caller's tree; the device leaf boxes get
   [0, 0] in the pad dims); wider is refused with MCG_EINVAL.
*/
enum {
  MCG_LIK_FLAT = 0,
  MCG_LIK_DIAG_GAUSS = 1,
  MCG_LIK_FULLCOV_GAUSS = 2,
  MCG_LIK_GAUSS_SHELL = 3,
  MCG_LIK_GAUSS_DATA = 4,
  MCG_LIK_CAUCHY_DATA = 5,
  MCG_LIK_GAUSS_MIX = 6
};
#define MCG_LIK_MIX_MAX 64

/* ---- prior kinds (replace the log_prior closure) ----
   FLAT     : (none)              lp = 0
   BOX      : lo[D], hi[D], lp_in lp = lp_in if lo <= x <= hi for all d (inclusive) else -inf
   OPEN_BOX : lo[D], hi[D], lp_in same with strict inequalities (test/nested_test.ml:23-28)
   DIAG_GAUSS: mu[D], sigma[D]    lp = Stats.log_multi_gaussian mu sigma x (stats.ml:98-108), in
                                  the canonical form of the DIAG_GAUSS likelihood (sigma > 0)
   Nested sampling takes a BOX / OPEN_BOX prior (draw_prior = uniform in [lo, hi],
   Stats.draw_uniform, stats.ml:126-128) or a DIAG_GAUSS prior (draw_prior = mu + sigma z per
   dim, Stats.draw_gaussian, stats.ml:113-124); with the Gaussian prior the walkers' constrained
   MH test log u < log_prior y - log_prior x (nested.ml:54-59) is a real test.  The reversible
   jump sampler (mcg_set_rjmcmc) takes every prior kind per model (lpa / lpb, mcmc.ml:116-118). */
enum { MCG_PRIOR_FLAT = 0, MCG_PRIOR_BOX = 1, MCG_PRIOR_OPEN_BOX = 2, MCG_PRIOR_DIAG_GAUSS = 3 };

/* ---- proposal kinds (replace jump_proposal / log_jump_prob, mcmc.mli:58-60) ----
   GAUSS        : s[1] or s[D]        y = x + s*z, z ~ N(0,1) per dim (symmetric)
   WRAP_UNIFORM : lo[D], hi[D], dx[D] Mcmc.uniform_wrapping per dim (mcmc.ml:187-196), symmetric
   KD_INTERP    : set with mcg_set_kd_proposal; independence proposal Interpolate_pdf.draw with
                  log_jump_prob _ y = log (jump_prob y)  (interpolate_pdf.ml:114-142)
   DE           : mode_hopping_frac; set with mcg_set_de_proposal (the sample array).
                  Mcmc.differential_evolution_proposal (mcmc.ml:198-218): y = x + d (s_j - s_i),
                  i != j uniform over the samples, d = 1.0 with probability mode_hopping_frac
                  (never drawn when it is 0) else N(0, 2.38/sqrt(2 ndim)); log_jump_prob = 0.
                  Also the proposal of nested sampling's walkers (nested.ml:53).
   MIXTURE      : Mcmc.combine_jump_proposals [(p_i, jp_i, ljp_i)] (mcmc.ml:165-185):
                  ncomp, then per component: p, comp_kind, ljp_mode, comp params, where
                    MCG_MIX_GAUSS         s[D]        y = x + s z, z ~ N(0, 1)
                    MCG_MIX_SHIFT_UNIFORM a[D], b[D]  y = x + random_between a b per dim
                                                     (the proposals of test/mcmc_test.ml)
                    MCG_MIX_WRAP_UNIFORM  lo, hi, dx  Mcmc.uniform_wrapping per dim
                    MCG_MIX_KD_INTERP     (none)      the context's kD tree (mcg_set_kd_proposal)
                  ljp_mode 0: the component's log_jump_prob is the constant 0 (what callers pass
                  for symmetric jumps); 1: its log density (GAUSS, SHIFT_UNIFORM; KD_INTERP is
                  always its density log q(y)).  Weights are normalised by their sum; the mixture
                  log_jump_prob folds log p_i + ljp_i with the reference's log(1 + exp) log-sum
                  (mcmc.ml:155-163).  A KD_INTERP component requires mcg_set_kd_proposal first
                  (which itself selects the plain KD proposal; set the MIXTURE after it).
                  Weights whose rounded normalised walk lets the largest uniform draw (1 - 2^-53)
                  pass every component are refused with MCG_EFAIL: the reference raises Failure
                  for such a draw (mcmc.ml:173), and the walk is monotone in the draw. */
enum { MCG_PROP_GAUSS = 1, MCG_PROP_WRAP_UNIFORM = 2, MCG_PROP_KD_INTERP = 3, MCG_PROP_DE = 4,
       MCG_PROP_MIXTURE = 5 };
enum { MCG_MIX_GAUSS = 1, MCG_MIX_SHIFT_UNIFORM = 2, MCG_MIX_WRAP_UNIFORM = 3,
       MCG_MIX_KD_INTERP = 4 };
#define MCG_MIX_MAX_COMPONENTS 8

/* ---- context ---- */
enum {
  MCG_FLAG_NESTED_FIXED_STOP = 1u << 0  /* use log(1/n) instead of the nested.ml:140 quirk */
};

typedef struct {
  int32_t device;          /* HIP device ordinal */
  uint32_t flags;          /* MCG_FLAG_* */
  uint64_t seed;           /* Philox key (replaces Random.init / self_init) */
  uint64_t chain_offset;   /* global id of this context's chain 0 (multi-GPU sharding) */
  int32_t lanes_per_chain; /* 0 = auto (1, 2, 4 or 8 lanes share one chain's dimensions) */
  int32_t steps_per_launch;/* 0 = auto (MH steps fused into one kernel launch) */
} mcg_opts;

typedef struct mcg_ctx mcg_ctx;

int mcg_ctx_create(mcg_ctx** out, const mcg_opts* opts);
void mcg_ctx_destroy(mcg_ctx* ctx);
const char* mcg_last_error(const mcg_ctx* ctx);
int mcg_abi_version(void);
/* name of the compiled device target ("gfx950") */
const char* mcg_device_arch(void);

/* ---- model descriptors ---- */
int mcg_set_likelihood(mcg_ctx* ctx, int32_t kind, int32_t ndim, const double* params, size_t n);
int mcg_set_prior(mcg_ctx* ctx, int32_t kind, const double* params, size_t n);
int mcg_set_proposal(mcg_ctx* ctx, int32_t kind, const double* params, size_t n);
/* Interpolate_pdf.make pts low high (interpolate_pdf.ml:111-112): kD tree built on the host
   with Kd_tree.tree_of_objects semantics (kd_tree.ml:155-175), flattened into HBM (at the model's
   padded width when ndim has no kD kernel of its own: see "Any ndim" above). */
int mcg_set_kd_proposal(mcg_ctx* ctx, const double* pts /*[M][D] row-major*/, int64_t M,
                        const double* low, const double* high);
/* Mcmc.differential_evolution_proposal ?mode_hopping_frac to_float from_float samples
   (mcmc.ml:198-218, mcmc.mli:215-218): samples [M][D] row-major (M >= 2: the reference's
   pick_samples never ends with one sample), kept in HBM; selects MCG_PROP_DE. */
int mcg_set_de_proposal(mcg_ctx* ctx, const double* samples, int64_t M, double mode_hopping_frac);

/* flattened tree of the last mcg_set_kd_proposal (pre-order; left child = node + 1):
   node_dim (-1 = leaf), node_split, node_right, node_leaf (-1 = internal), leaf_count,
   leaf_box [nleaves][2][D] (low then high), leaf_logq = log jump_prob inside the leaf */
int mcg_kd_info(mcg_ctx* ctx, int64_t* nnodes, int64_t* nleaves);
int mcg_kd_export(mcg_ctx* ctx, int32_t* node_dim, double* node_split, int32_t* node_right,
                  int32_t* node_leaf, int32_t* leaf_count, double* leaf_box, double* leaf_logq);

/* ---- chain state (like_prior / mcmc_sample records, mcmc.ml:17-25) ----
   x_soa [D][N]; ll, lp may be NULL -> evaluated on the device (mcmc.ml:59-61). */
int mcg_init(mcg_ctx* ctx, int64_t nchains, const double* x_soa, const double* ll,
             const double* lp);
int mcg_get_state(mcg_ctx* ctx, double* x_soa, double* ll, double* lp);
/* a counter that every entry point which may change the context's chains, model or RNG bumps
   (mcg_init, mcg_run, the mcg_set_* calls, mcg_nested, mcg_reseed, the RJ calls, ...): a host
   binding that keeps the chains device-resident between its own calls (the OCaml
   make_mcmc_sampler) skips the upload only while the token is the one it saw last */
uint64_t mcg_state_token(const mcg_ctx* ctx);

/* ---- Mcmc.mcmc_array (mcmc.ml:58-72) over every chain ----
   nbin burn-in steps, record 0 = post-burn-in state, then (n_rec-1)*nskip steps recording
   every nskip-th.  Records stay in device memory (read with mcg_get_records); with
   accumulate != 0 every recorded sample is folded into per-chain running statistics (Welford
   moments + log-space harmonic-mean partials) that mcg_stats reduces. */
typedef struct {
  int64_t nbin;
  int64_t nskip;
  int64_t n_rec;
  int32_t record_x;        /* keep x of recorded samples */
  int32_t record_llp;      /* keep ll, lp of recorded samples */
  int32_t record_accept;   /* keep the accept/reject bitmap of every step */
  int32_t accumulate;      /* fold recorded samples into running statistics */
  int32_t append;          /* continue the previous run's records/statistics: n_rec*nskip
                              steps, recording after every nskip-th (no initial record) */
} mcg_run_opts;

int mcg_run(mcg_ctx* ctx, const mcg_run_opts* opts);
/* rec_x [n_rec][D][N], rec_ll / rec_lp [n_rec][N], accept_bits [nsteps][ceil(N/64)] (bit c of
   row t = chain c accepted at step t of the last run).  Any pointer may be NULL. */
int mcg_get_records(mcg_ctx* ctx, double* rec_x, double* rec_ll, double* rec_lp,
                    uint64_t* accept_bits);
int64_t mcg_last_run_steps(const mcg_ctx* ctx);
/* lanes per chain the last MH run used (1, 2, 4 or 8; the auto choice or opts.lanes_per_chain) */
int mcg_last_run_lanes(const mcg_ctx* ctx);

/* ---- reversible-jump MCMC between two models (Mcmc.make_rjmcmc_sampler / rjmcmc_array,
   mcmc.ml:83-153) ----
   Each chain carries a model tag (0 = A, 1 = B) and a point of that model's dimension (padded
   with zeros to max(ndim_A, ndim_B) in the [Dmax][N] state).  A step draws u ~ U[0,1): with
   probability p_tag an internal jump of the current model, else a transition into the other
   model (mcmc.ml:92-102); log_jump_prob and the model log prior log p_m + lp_m follow
   mcmc.ml:103-118.  Likelihood kinds: FLAT, DIAG_GAUSS, GAUSS_SHELL, FULLCOV_GAUSS; priors as
   above.  Jump kinds (internal and into):
     MCG_RJ_JUMP_GAUSS       s[1] or s[D]   random walk y = x + s z, log_jump_prob 0
     MCG_RJ_JUMP_WRAP        lo, hi, dx     Mcmc.uniform_wrapping per dim, log_jump_prob 0
     MCG_RJ_JUMP_INDEP_GAUSS mu[D], s[D]    independence draw N(mu, s); log_jump_prob _ y =
                                            sum_d Stats.log_gaussian mu_d s_d y_d
     MCG_RJ_JUMP_KD          (kd_pts...)    independence draw Interpolate_pdf.draw from a kD tree
                                            over kd_pts; log_jump_prob _ y = log jump_prob y
   Transition proposals (into_kind) must be independence kinds (INDEP_GAUSS or KD): the
   reference's jintoa / jintob take the other model's point, which no descriptor kind uses. */
enum { MCG_RJ_JUMP_GAUSS = 1, MCG_RJ_JUMP_WRAP = 2, MCG_RJ_JUMP_INDEP_GAUSS = 3, MCG_RJ_JUMP_KD = 4 };

typedef struct {
  int32_t ndim;
  int32_t lik_kind;   const double* lik_params;   size_t n_lik;
  int32_t prior_kind; const double* prior_params; size_t n_prior;
  int32_t jump_kind;  const double* jump_params;  size_t n_jump;   /* internal jump (jpa, ljpa) */
  int32_t into_kind;  const double* into_params;  size_t n_into;   /* jump into this model (jintoa, ljpintoa) */
  const double* kd_pts; int64_t kd_M;              /* [M][ndim] tree points for the KD kinds */
  const double* kd_low; const double* kd_high;     /* tree bounds (Interpolate_pdf.make) */
  double model_prior;                              /* pa / pb (pa + pb = 1, mcmc.ml:90) */
} mcg_rj_model;

int mcg_set_rjmcmc(mcg_ctx* ctx, const mcg_rj_model* a, const mcg_rj_model* b);
/* model[N] (0 = A, 1 = B) or NULL for rjmcmc_array's fair coin per chain (mcmc.ml:123);
   xa [ndim_A][N], xb [ndim_B][N]: the start point of each chain in model A and in model B (the
   (a, b) pair of rjmcmc_array, per chain); the chain starts from the one of its model.  ll / lp
   are evaluated on the device (lp includes log p_model, mcmc.ml:126-128).  Then mcg_run runs
   rjmcmc_array's schedule (mcmc.ml:129-139) over every chain; the state and records use the
   padded [Dmax][N] layout (dims beyond the chain's model are 0). */
int mcg_rj_init(mcg_ctx* ctx, int64_t nchains, const uint8_t* model, const double* xa, const double* xb);
/* model tags: current state [N] and recorded samples [n_rec][N] of the last run (any may be
   NULL); counts = rjmcmc_model_counts over every recorded sample of every chain (mcmc.ml:141-149) */
int mcg_rj_get_models(mcg_ctx* ctx, uint8_t* state_model, uint8_t* rec_model);
int mcg_rj_model_counts(mcg_ctx* ctx, uint64_t* na, uint64_t* nb);

/* ---- counters (mcmc.ml:27-35) ---- */
int mcg_get_counters(mcg_ctx* ctx, uint64_t* naccept, uint64_t* nreject);
int mcg_reset_counters(mcg_ctx* ctx);

/* ---- reductions over the recorded samples of the last run ----
   Tile partials: 256-chain tiles reduced on the device by a fixed pairwise tree (layout per
   tile: n, mean[D], m2[D], hm_max, hm_sum; 2D+3 doubles).  Tiles are independent of the GPU
   count, so an all-gather of every rank's tiles followed by mcg_combine_tiles gives
   bit-identical results on 1/2/4/8 GPUs. */
int64_t mcg_num_tiles(const mcg_ctx* ctx);
int mcg_tile_stats(mcg_ctx* ctx, double* tiles /*[ntiles][2D+3]*/);
/* device pointer of the tile partials (for a device-side all-gather, e.g. RCCL); the tile
   kernel is enqueued on the context's stream (mcg_sync before another stream reads them) */
int mcg_tile_stats_device(mcg_ctx* ctx, void** dev_ptr, int64_t* ntiles);
/* the tile partials written straight into a caller-owned device buffer of at least
   mcg_num_tiles(ctx) x (2D+3) doubles on the context's device (e.g. the send buffer of an RCCL
   all-gather), complete when this returns */
int mcg_tile_stats_into(mcg_ctx* ctx, double* dev_tiles);
/* Stats.multi_mean / multi_std (stats.ml:58-87, std with n-1) and the harmonic-mean evidence
   (evidence.ml:101-107) in log space: log Z = log n - logsumexp(-ll). */
int mcg_combine_tiles(int32_t ndim, int64_t ntiles, const double* tiles, double* mean, double* sd,
                      double* log_z_hm);
/* single-context convenience: tiles + combine */
int mcg_stats(mcg_ctx* ctx, double* mean, double* sd, double* log_z_hm);

/* ---- Nested.nested_evidence (nested.ml:122-146) ----
   Uses the context's likelihood and (box) prior; the DE proposal (mcmc.ml:198-218) runs inside.
   k = live points retired per generation (k = 1 is the reference algorithm; k > 1 runs k
   constrained walkers in parallel and shrinks the volume with live counts n, n-1, ..., n-k+1). */
typedef struct {
  int64_t nlive;          /* default 1000 */
  int64_t nmcmc;          /* default 1000 */
  int64_t k;              /* default 1 */
  double epsrel;          /* default 0.01 */
  double mode_hop;        /* default 0.1 */
  int64_t max_dead;       /* safety cap (0 = 1000 * nlive) */
} mcg_nested_opts;

typedef struct {
  double log_ev;
  double log_dev;
  int64_t n_dead;
  int64_t n_total;        /* n_dead + nlive */
  int64_t n_gen;
  int32_t converged;      /* 1: remaining_integral_negligable fired (nested.ml:45-48, 144);
                             0: the max_dead cap ended the run first -- log_ev / log_dev /
                             weights then come from an unconverged run */
} mcg_nested_result;

/* observer: called after each batch of generations with the newly retired points (batch form
   of the per-point ?observer of nested.ml:136); may be NULL. */
typedef void (*mcg_observer_fn)(void* user, const double* pts /*[n][D]*/, const double* ll,
                                const double* lp, int64_t n);

int mcg_nested(mcg_ctx* ctx, const mcg_nested_opts* opts, mcg_nested_result* res,
               mcg_observer_fn observer, void* user);
/* all points of the last nested run (dead in retirement order, then live ascending in ll):
   pts [n_total][D] row-major, ll, lp, log_wts [n_total] (nested_output, nested.ml:20) */
int mcg_nested_get(mcg_ctx* ctx, double* pts, double* ll, double* lp, double* log_wts);
/* The last nested run's ll, lp and log_wts [n_total] (as mcg_nested_get writes them) handed to
   the caller without a copy: three malloc'd arrays the caller owns and releases with mcg_free.
   Afterwards mcg_nested_get still copies the points (pts) but refuses ll / lp / log_wts
   (MCG_ESTATE) until the next run.  The context then allocates the next run's host blocks,
   sized like this run's, and prefaults them in the background (about 24 bytes per point of this
   run stay resident until the next run or mcg_destroy).  (No reference counterpart:
   nested_output's arrays are fresh OCaml arrays, nested.ml:20, which this gives a binding
   without a second copy.) */
int mcg_nested_take(mcg_ctx* ctx, double** ll, double** lp, double** log_wts);
void mcg_free(void* p);
/* The last nested run's points as rows in a caller-owned device buffer on the context's device
   (the send buffer of a replica all-gather over RCCL), device to device: row i of
   [n_total] = (pts[i][0..D) when with_points, ll[i], lp[i]), `row_stride` doubles apart
   (>= D + 2 with points, >= 2 without), in nested_output order.  Complete when this returns.
   Replaces nested_output's host copy for the exchange: only the gathered rows of every
   replica come back to the host, for mcg_nested_merge. */
int mcg_nested_rows_into(mcg_ctx* ctx, double* dev_rows, int64_t row_stride, int32_t with_points);
/* Nested.log_total_error_estimate (nested.ml:148-150) */
double mcg_log_total_error_estimate(double log_ev, double log_dev, int64_t nlive);
/* Nested.posterior_samples n (nested.ml:167-178) as indices: the running sums of exp log_wts
   (sequential, glibc exp: :170-173) and, per draw, Random.float 1.0 -> weight_binary_search_index
   (:152-165) on the device.  Draw i of a call takes u53 of Philox counter (i lo, i hi, call, tag 5):
   `call` counts this context's posterior_samples calls since mcg_ctx_create / mcg_reseed, so
   repeated calls draw new samples, as the reference's global Random state does.  idx [n] gets
   the index into the npts points of each draw. */
int mcg_posterior_samples(mcg_ctx* ctx, const double* log_wts, int64_t npts, int64_t n, int64_t* idx);

/* ---- nested replicas: merge independent runs into one (multi-GPU C3) ----
   Each of nruns independent runs (one per GPU) gives its points in nested_output order (dead in
   retirement order, then the final live points ascending; nested.ml:143), concatenated run
   after run in ll.  Run r retired its i-th dead point with nlive[r] - (i mod k[r]) live points
   and its j-th final live point with nlive[r] - j (the final live points retired one by one).
   The merged run visits every point in ascending ll (ties: run, then index) with the live
   count n_p = the sum over runs of each run's count at level ll_p; volumes shrink by
   log1p(-1/n_p) and the trapezoid rule of evidence_error_and_weights (nested.ml:81-120) gives
   log Z, log dZ and the log weights.  order[p] = index into the concatenation of the p-th
   merged point; log_wts is in merged order.  With equal runs of nlive/R points this is one run
   of nlive points. */
int mcg_nested_merge(int32_t nruns, const int64_t* n_total, const int64_t* nlive, const int64_t* k,
                     const double* ll, int64_t* order, double* log_ev, double* log_dev,
                     double* log_wts);

/* ---- evidence_error_and_weights (nested.ml:81-120) on the host ----
   The fold mcg_nested runs beside the GPU, over a caller's points in nested_output order: ll
   [ntot], the ntot - nlive dead points in retirement order then the nlive final live points
   ascending; dead point i was retired with nlive - (i mod k) live points (k retirements per
   generation; k = 1 is the reference's loop).  Writes log Z, log dZ and the normalised log
   weights [ntot]: the same bits as mcg_nested's own (and the oracle's or_evidence_weights).
   chunk > 0 streams the dead points in chunks of that many points first, as mcg_nested does
   while the GPU runs (the result does not depend on the chunking); 0 folds everything at once.
   Returns MCG_EINVAL unless 1 <= k < nlive <= ntot (as mcg_nested: retiring every live point in
   one generation leaves no volume). */
int mcg_evidence_weights(int64_t ntot, int64_t nlive, int64_t k, const double* ll, int64_t chunk,
                         double* log_ev, double* log_dev, double* log_wts);

/* ---- kD-tree evidence integrals over samples (Evidence.Make(MO), evidence.ml:66-221) ----
   pts [n][ndim] row-major, ll, lp [n]: one sample array (several chains: concatenated).
   evidence_direct ?n (evidence.ml:145-156): duplicates removed, kD tree of the samples
   (kd_tree.ml:155-175), cells with fewer than nbox samples, sum of cell volume x mean posterior.
   evidence_lebesgue ?n ?eps (evidence.ml:194-221): samples up to the first gap > eps in 1/L,
   prior mass of their cells (median prior) / mean 1/L.  Host computation; deterministic. */
int mcg_evidence_direct(int32_t ndim, int64_t n, const double* pts, const double* ll, const double* lp,
                        int64_t nbox, double* out);
int mcg_evidence_lebesgue(int32_t ndim, int64_t n, const double* pts, const double* ll, const double* lp,
                          int64_t nbox, double eps, double* out);

/* ---- Read_write text formats (read_write.ml:19-101) ----
   A Read_write file is rows of doubles printed with OCaml Printf "%g" (C %g; nan prints as
   "nan"), separated by single spaces, one row per line:
     write / write_sample (read_write.ml:19-30): coords..., log_likelihood, log_prior
     write_nested (read_write.ml:58-66): a "log_ev log_dev" first line, then
                                         coords..., log_likelihood, log_prior, log_weight
   mcg_write_rows writes `header` (may be NULL, e.g. the write_nested first line) and then
   rows [nrows][ncols] (formatted in parallel, written in order); append != 0 appends.
   mcg_read_rows_shape counts the non-blank lines after skip_lines and their common field count
   (ragged rows -> MCG_EFAIL); mcg_read_rows parses them (Scanf " %g ", read_write.ml:33-56) into
   rows [nrows][ncols] and, if header != NULL, the first nheader fields of line 0. */
int mcg_write_rows(const char* path, int32_t append, const char* header, int64_t nrows, int32_t ncols,
                   const double* rows);
int mcg_read_rows_shape(const char* path, int64_t skip_lines, int64_t* nrows, int32_t* ncols);
int mcg_read_rows(const char* path, int64_t skip_lines, int64_t nrows, int32_t ncols, double* rows,
                  double* header, int32_t nheader);

/* ---- device timing of the dominant kernel (HIP events on the launch stream) ---- */
typedef struct {
  int64_t launches;
  double total_ms;
  double last_ms;
} mcg_kernel_timing;
int mcg_get_kernel_timing(mcg_ctx* ctx, const char* kernel, mcg_kernel_timing* out);
int mcg_set_timing(mcg_ctx* ctx, int32_t enabled);
/* synchronize the context's stream */
int mcg_sync(mcg_ctx* ctx);
/* Random.init seed (the reference's global RNG state, mcmc.ml:49): set the Philox key and restart
   the context's step counter at 0.  Without it the counter runs on across mcg_init / mcg_run /
   mcg_rj_init, so repeated runs on one context never replay a draw. */
int mcg_reseed(mcg_ctx* ctx, uint64_t seed);
/* the Philox step index the next MH step will draw at */
uint64_t mcg_rng_step(const mcg_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
