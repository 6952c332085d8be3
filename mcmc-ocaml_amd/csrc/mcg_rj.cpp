// mcg_rj.cpp -- host side of the reversible-jump sampler (Mcmc.make_rjmcmc_sampler /
// rjmcmc_array / rjmcmc_model_counts, mcmc.ml:83-153): packs the two model descriptors into
// the padded device layout of mcg_rj_kernel.h, builds the models' kD trees, starts the chains.
// mcg_run drives the steps (mcg_runtime.cpp dispatches to the RJ kernel when rj_active).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "mcg_runtime.h"

using namespace mcg;

namespace {

const double kNegHalfLog2Pi = -0.91893853320467274178;

int pack_jump(mcg_ctx* ctx, int32_t kind, int D, int DM, const double* p, size_t n, bool into,
              bool has_tree, std::vector<double>& o) {
  o.clear();
  if (into && kind != MCG_RJ_JUMP_INDEP_GAUSS && kind != MCG_RJ_JUMP_KD)
    return set_error(ctx, MCG_EINVAL, "RJ: the jump into a model must be INDEP_GAUSS or KD");
  switch (kind) {
    case MCG_RJ_JUMP_GAUSS:
      if (!p || (n != 1 && n != (size_t)D)) return set_error(ctx, MCG_EINVAL, "RJ GAUSS jump: s[1] or s[D]");
      o.assign(DM, 0.0);
      for (int d = 0; d < D; ++d) o[d] = p[n == 1 ? 0 : d];
      return MCG_OK;
    case MCG_RJ_JUMP_WRAP:
      if (!p || n != 3 * (size_t)D) return set_error(ctx, MCG_EINVAL, "RJ WRAP jump: lo[D], hi[D], dx[D]");
      o.assign(3 * (size_t)DM, 0.0);
      for (int d = 0; d < D; ++d) { o[d] = p[d]; o[DM + d] = p[D + d]; o[2 * DM + d] = p[2 * D + d]; }
      return MCG_OK;
    case MCG_RJ_JUMP_INDEP_GAUSS: {
      if (!p || n != 2 * (size_t)D) return set_error(ctx, MCG_EINVAL, "RJ INDEP_GAUSS jump: mu[D], s[D]");
      o.assign(4 * (size_t)DM + 1, 0.0);
      double C = 0.0;
      for (int d = 0; d < D; ++d) {
        if (!(p[D + d] > 0.0)) return set_error(ctx, MCG_EINVAL, "RJ INDEP_GAUSS jump: s > 0");
        o[d] = p[d];
        o[DM + d] = p[D + d];
        o[2 * DM + d] = 1.0 / p[D + d];
        o[3 * DM + d] = p[d] * o[2 * DM + d];
        C = C + (kNegHalfLog2Pi - std::log(p[D + d]));   // Stats.log_gaussian (stats.ml:98-101)
      }
      o[4 * DM] = C;
      return MCG_OK;
    }
    case MCG_RJ_JUMP_KD:
      if (!has_tree) return set_error(ctx, MCG_EINVAL, "RJ KD jump: the model needs kd_pts");
      o.assign(1, 0.0);
      return MCG_OK;
    default:
      return set_error(ctx, MCG_EINVAL, "RJ: unknown jump kind %d", kind);
  }
}

}  // namespace

extern "C" {

int mcg_set_rjmcmc(mcg_ctx* ctx, const mcg_rj_model* a, const mcg_rj_model* b) {
  if (!ctx || !a || !b) return MCG_EINVAL;
  const mcg_rj_model* m[2] = {a, b};
  if (!(std::fabs(a->model_prior + b->model_prior - 1.0) < std::sqrt(2.220446049250313e-16)) ||
      !(a->model_prior > 0.0) || !(b->model_prior > 0.0))
    return set_error(ctx, MCG_EINVAL, "RJ: model priors pa + pb must be 1 (mcmc.ml:90)");
  const int DM = std::max(a->ndim, b->ndim);
  if (a->ndim < 1 || b->ndim < 1) return set_error(ctx, MCG_EINVAL, "RJ: ndim >= 1");
  if (!find_rj_kernel(DM)) return set_error(ctx, MCG_EINVAL, "RJ: no compiled kernel for max ndim %d", DM);
  (void)hipSetDevice(ctx->opts.device);
  // fold_counters zeroes the device tallies too: a validation error below leaves consistent counters
  int qrc;
  if ((qrc = quiesce(ctx)) || (qrc = fold_counters(ctx))) return qrc;
  std::vector<double> dev(32, 0.0);
  int rc;
  for (int k = 0; k < 2; ++k) {
    const mcg_rj_model* q = m[k];
    const int D = q->ndim;
    if (q->lik_kind != MCG_LIK_FLAT && q->lik_kind != MCG_LIK_DIAG_GAUSS && q->lik_kind != MCG_LIK_GAUSS_SHELL &&
        q->lik_kind != MCG_LIK_FULLCOV_GAUSS)
      return set_error(ctx, MCG_EINVAL, "RJ: likelihood kind %d not supported", q->lik_kind);
    std::vector<double> lik, pri, jmp, into;
    if ((rc = pack_likelihood(ctx, q->lik_kind, D, q->lik_params, q->n_lik, lik, nullptr, nullptr))) return rc;
    if ((rc = pack_prior(ctx, q->prior_kind, D, q->prior_params, q->n_prior, pri))) return rc;
    const bool tree = q->kd_pts && q->kd_M > 0 && q->kd_low && q->kd_high;
    if ((rc = pack_jump(ctx, q->jump_kind, D, DM, q->jump_params, q->n_jump, false, tree, jmp))) return rc;
    if ((rc = pack_jump(ctx, q->into_kind, D, DM, q->into_params, q->n_into, true, tree, into))) return rc;
    if (tree) {
      if ((rc = kd_build(ctx, q->kd_pts, q->kd_M, D, q->kd_low, q->kd_high, &ctx->rj_kd[k]))) return rc;
      // root box padded to DM (the descent tests every one of the DM coordinates)
      std::vector<double>& root = ctx->rj_root[k];
      root.assign(2 * (size_t)DM, 0.0);
      for (int d = 0; d < DM; ++d) {
        root[d] = d < D ? q->kd_low[d] : -HUGE_VAL;
        root[DM + d] = d < D ? q->kd_high[d] : HUGE_VAL;
      }
      if ((rc = hip_check(ctx, ctx->d_rj_root[k].ensure(root.size() * 8), "alloc rj root"))) return rc;
      if ((rc = hip_check(ctx, hipMemcpy(ctx->d_rj_root[k].p, root.data(), root.size() * 8, hipMemcpyHostToDevice), "copy rj root"))) return rc;
    } else {
      ctx->rj_kd[k].built = false;
    }
    double* h = &dev[16 * (size_t)k];
    h[0] = D;
    h[1] = std::log(q->model_prior);
    h[2] = q->model_prior;
    h[3] = q->lik_kind;
    h[4] = q->prior_kind;
    h[5] = q->jump_kind;
    h[6] = q->into_kind;
    auto put = [&](const std::vector<double>& blk) {
      const double off = (double)dev.size();
      dev.insert(dev.end(), blk.begin(), blk.end());
      return off;
    };
    const std::vector<double> plik = pad_lik(q->lik_kind, D, DM, lik);
    // (dev grows below: re-take the header pointer afterwards)
    const std::vector<double> ppri = q->prior_kind == MCG_PRIOR_DIAG_GAUSS ? pad_gauss_prior(D, DM, pri)
                                                                         : pad_prior(D, DM, pri, -HUGE_VAL, HUGE_VAL);
    const double o_lik = put(plik), o_pri = put(ppri), o_j = put(jmp), o_i = put(into);
    double* hh = &dev[16 * (size_t)k];
    hh[7] = o_lik; hh[8] = o_pri; hh[9] = o_j; hh[10] = o_i;
  }
  ctx->rj_host = dev;
  if ((rc = hip_check(ctx, ctx->d_rj.ensure(dev.size() * 8), "alloc rj"))) return rc;
  if ((rc = hip_check(ctx, hipMemcpy(ctx->d_rj.p, dev.data(), dev.size() * 8, hipMemcpyHostToDevice), "copy rj"))) return rc;
  ctx->D = DM;
  ctx->Dk = DM;
  ctx->lik_kind = MCG_LIK_FLAT;
  ctx->rj_active = true;
  ctx->N = 0;
  return MCG_OK;
}

int mcg_rj_init(mcg_ctx* ctx, int64_t nchains, const uint8_t* model, const double* xa, const double* xb) {
  if (!ctx || nchains < 1 || !xa || !xb) return MCG_EINVAL;
  if (!ctx->rj_active) return set_error(ctx, MCG_ESTATE, "mcg_rj_init before mcg_set_rjmcmc");
  if (nchains > (int64_t)0x7FFFFFFF) return set_error(ctx, MCG_EINVAL, "too many chains");
  (void)hipSetDevice(ctx->opts.device);
  const int DM = ctx->D;
  const size_t N = (size_t)nchains;
  int rc;
  if ((rc = quiesce(ctx)) || (rc = fold_counters(ctx))) return rc;
  if ((rc = hip_check(ctx, ctx->d_x.ensure(N * DM * 8), "alloc x"))) return rc;
  if ((rc = hip_check(ctx, ctx->d_ll.ensure(N * 8), "alloc ll"))) return rc;
  if ((rc = hip_check(ctx, ctx->d_lp.ensure(N * 8), "alloc lp"))) return rc;
  if ((rc = hip_check(ctx, ctx->d_nacc.ensure(N * 8), "alloc counters"))) return rc;
  if ((rc = hip_check(ctx, ctx->d_tag.ensure(N), "alloc tags"))) return rc;
  if ((rc = hip_check(ctx, ctx->d_rj_nb.ensure(N * 8), "alloc rj counts"))) return rc;
  if ((rc = hip_check(ctx, hipMemset(ctx->d_nacc.p, 0, N * 8), "zero counters"))) return rc;
  const int DA = (int)ctx->rj_host[0], DB = (int)ctx->rj_host[16];
  DevBuf dxa, dxb;
  if ((rc = hip_check(ctx, dxa.ensure(N * DA * 8), "alloc xa"))) return rc;
  if ((rc = hip_check(ctx, dxb.ensure(N * DB * 8), "alloc xb"))) return rc;
  if ((rc = hip_check(ctx, hipMemcpy(dxa.p, xa, N * DA * 8, hipMemcpyHostToDevice), "copy xa"))) return rc;
  if ((rc = hip_check(ctx, hipMemcpy(dxb.p, xb, N * DB * 8, hipMemcpyHostToDevice), "copy xb"))) return rc;
  if ((rc = hip_check(ctx, hipMemset(ctx->d_rj_nb.p, 0, N * 8), "zero rj counts"))) return rc;
  if (model) {
    for (size_t i = 0; i < N; ++i)
      if (model[i] > 1) return set_error(ctx, MCG_EINVAL, "RJ: model tags are 0 (A) or 1 (B)");
    if ((rc = hip_check(ctx, hipMemcpy(ctx->d_tag.p, model, N, hipMemcpyHostToDevice), "copy tags"))) return rc;
  }
  ctx->N = nchains;
  // the Philox step counter runs on (mcg_init); the start coin draws at the current step
  ctx->last_nsteps = 0;
  ctx->nrec_total = 0;
  ctx->rec_stored = 0;
  MhArgs a = base_args(ctx);
  a.step_base = ctx->steps_done;
  if ((rc = hip_check(ctx, find_rj_init(DM)(a, model ? 0 : 1, (const double*)dxa.p, (const double*)dxb.p,
                                            ctx->stream), "rj init launch"))) return rc;
  return hip_check(ctx, hipStreamSynchronize(ctx->stream), "rj init sync");
}

int mcg_rj_get_models(mcg_ctx* ctx, uint8_t* state_model, uint8_t* rec_model) {
  if (!ctx) return MCG_EINVAL;
  if (!ctx->rj_active || ctx->N < 1) return set_error(ctx, MCG_ESTATE, "no reversible-jump chains");
  int rc;
  if ((rc = hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync"))) return rc;
  const size_t N = (size_t)ctx->N;
  if (state_model && (rc = hip_check(ctx, hipMemcpy(state_model, ctx->d_tag.p, N, hipMemcpyDeviceToHost), "copy tags"))) return rc;
  if (rec_model) {
    if (!ctx->rec_llp_valid) return set_error(ctx, MCG_ESTATE, "last run did not record ll/lp (tags ride with them)");
    if ((rc = hip_check(ctx, hipMemcpy(rec_model, ctx->d_rec_tag.p, (size_t)ctx->rec_stored * N, hipMemcpyDeviceToHost), "copy rec tags"))) return rc;
  }
  return MCG_OK;
}

int mcg_rj_model_counts(mcg_ctx* ctx, uint64_t* na, uint64_t* nb) {
  if (!ctx || !na || !nb) return MCG_EINVAL;
  if (!ctx->rj_active || ctx->N < 1) return set_error(ctx, MCG_ESTATE, "no reversible-jump chains");
  int rc;
  if ((rc = hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync"))) return rc;
  std::vector<unsigned long long> c((size_t)ctx->N);
  if ((rc = hip_check(ctx, hipMemcpy(c.data(), ctx->d_rj_nb.p, c.size() * 8, hipMemcpyDeviceToHost), "copy rj counts"))) return rc;
  uint64_t b = 0;
  for (auto v : c) b += v;
  const uint64_t tot = (uint64_t)ctx->nrec_total * (uint64_t)ctx->N;
  *nb = b;
  *na = tot - b;
  return MCG_OK;
}

}  // extern "C"

namespace mcg {

// the RJ fields of MhArgs (trees, tags, descriptor)
void rj_args(mcg_ctx* ctx, MhArgs& a) {
  a.rj = (const double*)ctx->d_rj.p;
  a.tag = (uint8_t*)ctx->d_tag.p;
  a.rec_tag = (uint8_t*)ctx->d_rec_tag.p;
  a.rj_nb = (unsigned long long*)ctx->d_rj_nb.p;
  for (int k = 0; k < 2; ++k) {
    const KdState& t = ctx->rj_kd[k];
    a.rj_kd[k].nodes = (const KdNode*)t.d_nodes.p;
    a.rj_kd[k].logq = (const double*)t.d_logq.p;
    a.rj_kd[k].box = (const double*)t.d_box.p;
    a.rj_kd[k].root = (const double*)ctx->d_rj_root[k].p;
    a.rj_kd[k].pt_leaf = (const int32_t*)t.d_pt_leaf.p;
    a.rj_kd[k].M = t.M;
  }
}

}  // namespace mcg
