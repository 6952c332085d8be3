// mcg_runtime.cpp -- host runtime behind the C-ABI (include/mcg.h).
//
// Owns the HIP device buffers of a sampling context, turns the reference's closure arguments
// (mcmc.mli:58-60) into device constant blocks, slices Mcmc.mcmc_array (mcmc.ml:58-72) into
// fused multi-step kernel launches, and finishes the tile reductions.  Nested sampling lives in
// mcg_nested.cpp, the kD tree build in mcg_kdtree.cpp.
#include "mcg_runtime.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace mcg;

namespace mcg {

int set_error(mcg_ctx* ctx, int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  return code;
}

int hip_check(mcg_ctx* ctx, hipError_t e, const char* what) {
  if (e == hipSuccess) return MCG_OK;
  return set_error(ctx, e == hipErrorOutOfMemory ? MCG_ENOMEM : MCG_EDEVICE, "%s: %s", what,
                   hipGetErrorString(e));
}

// Host-side writes to context buffers (blocking copies, frees) do not order against the
// context's non-blocking stream: every entry point that rewrites them drains the stream first.
int quiesce(mcg_ctx* ctx) {
  ++ctx->state_token;                 // every entry point that may change the context's state
  if (!ctx->stream) return MCG_OK;
  return hip_check(ctx, hipStreamSynchronize(ctx->stream), "drain context stream");
}

// Fold the per-chain device accept counters of the current chains into the context totals
// (acc_base / rej_base), zero the step tally AND the device counters, so the context stays
// consistent whatever the caller does next (an entry point that fails after the fold must not
// leave the device tallies to be counted twice).  The caller has drained the stream.
int fold_counters(mcg_ctx* ctx) {
  if (ctx->N < 1 || !ctx->d_nacc.p || ctx->nsteps_total == 0) {
    ctx->nsteps_total = 0;
    return MCG_OK;
  }
  std::vector<uint64_t> h((size_t)ctx->N);
  int rc = hip_check(ctx, hipMemcpy(h.data(), ctx->d_nacc.p, h.size() * 8, hipMemcpyDeviceToHost), "copy counters");
  if (rc) return rc;
  if ((rc = hip_check(ctx, hipMemset(ctx->d_nacc.p, 0, h.size() * 8), "zero counters"))) return rc;
  uint64_t s = 0;
  for (uint64_t v : h) s += v;
  ctx->acc_base += s;
  ctx->rej_base += (uint64_t)ctx->nsteps_total * (uint64_t)ctx->N - s;
  ctx->nsteps_total = 0;
  return MCG_OK;
}

DevBuf::~DevBuf() { release(); }
void DevBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
}
hipError_t DevBuf::ensure(size_t n) {
  if (n <= bytes && p) return hipSuccess;
  release();
  if (n == 0) n = 8;
  hipError_t e = hipMalloc(&p, n);
  if (e != hipSuccess) {
    p = nullptr;
    return e;
  }
  bytes = n;
  return hipSuccess;
}

// portable exp for x <= 0 (same operation sequence as the device pexp)
double host_pexp(double x) {
  if (!(x > -708.0)) return 0.0;
  const double inv_ln2 = 0x1.71547652b82fep+0;
  const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
  double kd = std::floor(std::fma(x, inv_ln2, 0.5));
  double r = std::fma(-kd, ln2_hi, x);
  r = std::fma(-kd, ln2_lo, r);
  static const double c[] = {0x1.ae64567f544e4p-26, 0x1.27e4fb7789f5cp-22, 0x1.71de3a556c734p-19,
                             0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-13, 0x1.6c16c16c16c17p-10,
                             0x1.1111111111111p-7,  0x1.5555555555555p-5,  0x1.5555555555555p-3,
                             0.5, 1.0, 1.0};
  double p = 0x1.1eed8eff8d898p-29;
  for (double ci : c) p = std::fma(p, r, ci);
  uint64_t sc = (uint64_t)((int)kd + 1023) << 52;
  double scale;
  std::memcpy(&scale, &sc, 8);
  return p * scale;
}

void timing_begin(mcg_ctx* ctx, hipEvent_t* a, hipEvent_t* b) {
  for (hipEvent_t* e : {a, b}) {
    if (!ctx->ev_free.empty()) {
      *e = ctx->ev_free.back();
      ctx->ev_free.pop_back();
    } else if (hipEventCreate(e) != hipSuccess) {
      *e = nullptr;
    }
  }
  if (*a) (void)hipEventRecord(*a, ctx->stream);
}

void timing_end(mcg_ctx* ctx, hipEvent_t a, hipEvent_t b, int kind) {
  if (!a || !b) return;
  (void)hipEventRecord(b, ctx->stream);
  ctx->ev_pending.push_back(mcg_ctx::Pending{a, b, kind});
}

void timing_harvest(mcg_ctx* ctx) {
  for (auto& p : ctx->ev_pending) {
    (void)hipEventSynchronize(p.b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, p.a, p.b);
    mcg_kernel_timing& t = p.kind == 0 ? ctx->t_mh : ctx->t_walk;
    t.launches += 1;
    t.total_ms += ms;
    t.last_ms = ms;
    ctx->ev_free.push_back(p.a);
    ctx->ev_free.push_back(p.b);
  }
  ctx->ev_pending.clear();
}

}  // namespace mcg

static const double kNegHalfLog2Pi = -0.91893853320467274178;

// Mcmc.combine_jump_proposals (mcmc.ml:165-185) -> device layout (mcg_mh_kernel.h MixLayout):
// [ncomp] then per component (stride 5 + 3D): p / ptot, log(p / ptot), comp kind, ljp mode,
// constant C of the component log density, then 3D parameters:
//   GAUSS: s[D], 1/s[D]  (C = sum_d (-1/2 log 2pi - log s_d))
//   SHIFT_UNIFORM: a[D], b[D], b - a[D]  (C = -sum_d log(b_d - a_d))
//   WRAP_UNIFORM: lo[D], hi[D], dx[D]
// (at the kernel width Dk: padded dims get zero steps, zero bounds and no density term)
static int pack_mixture(mcg_ctx* ctx, const double* params, size_t n, std::vector<double>& dev) {
  const int D = ctx->D, Dk = ctx->Dk;
  if (!params || n < 1) return mcg::set_error(ctx, MCG_EINVAL, "MIXTURE: ncomp, components...");
  const int nc = (int)params[0];
  if (nc < 1 || nc > MCG_MIX_MAX_COMPONENTS || (double)nc != params[0])
    return mcg::set_error(ctx, MCG_EINVAL, "MIXTURE: 1 <= ncomp <= %d", MCG_MIX_MAX_COMPONENTS);
  const size_t stride = 5 + 3 * (size_t)Dk;
  dev.assign(1 + nc * stride, 0.0);
  dev[0] = nc;
  double ptot = 0.0;
  size_t o = 1;
  for (int c = 0; c < nc; ++c) {               // first pass: validate, sum the weights
    if (o + 3 > n) return mcg::set_error(ctx, MCG_EINVAL, "MIXTURE: component %d truncated", c);
    const double p = params[o];
    const int ck = (int)params[o + 1], mode = (int)params[o + 2];
    size_t np = ck == MCG_MIX_GAUSS ? D : ck == MCG_MIX_SHIFT_UNIFORM ? 2 * D
              : ck == MCG_MIX_WRAP_UNIFORM ? 3 * D : ck == MCG_MIX_KD_INTERP ? 0 : (size_t)-1;
    if (np == (size_t)-1) return mcg::set_error(ctx, MCG_EINVAL, "MIXTURE: unknown component kind %d", ck);
    if (!(p >= 0.0) || (mode != 0 && mode != 1))
      return mcg::set_error(ctx, MCG_EINVAL, "MIXTURE: component %d needs p >= 0, ljp_mode 0/1", c);
    if (ck == MCG_MIX_WRAP_UNIFORM && mode == 1)
      return mcg::set_error(ctx, MCG_EINVAL, "MIXTURE: the wrapping-uniform density is symmetric; use ljp_mode 0");
    if (ck == MCG_MIX_KD_INTERP && !ctx->kd.built)
      return mcg::set_error(ctx, MCG_ESTATE, "MIXTURE: KD_INTERP component needs mcg_set_kd_proposal first");
    if (o + 3 + np > n) return mcg::set_error(ctx, MCG_EINVAL, "MIXTURE: component %d truncated", c);
    ptot = ptot + p;                            // List.fold_left (+.) 0.0 (mcmc.ml:166)
    o += 3 + np;
  }
  if (o != n) return mcg::set_error(ctx, MCG_EINVAL, "MIXTURE: %zu trailing parameters", n - o);
  if (!(ptot > 0.0)) return mcg::set_error(ctx, MCG_EINVAL, "MIXTURE: weights sum to zero");
  o = 1;
  for (int c = 0; c < nc; ++c) {
    double* q = &dev[1 + c * stride];
    const int ck = (int)params[o + 1], mode = (int)params[o + 2];
    const double* u = params + o + 3;
    q[0] = params[o] / ptot;                    // mcmc.ml:167
    q[1] = std::log(q[0]);                      // log p, mcmc.ml:178
    q[2] = ck;
    q[3] = ck == MCG_MIX_KD_INTERP ? 1 : mode;
    double C = 0.0;
    if (ck == MCG_MIX_GAUSS) {
      for (int d = 0; d < D; ++d) {
        if (!(u[d] > 0.0)) return mcg::set_error(ctx, MCG_EINVAL, "MIXTURE: GAUSS scale must be > 0");
        q[5 + d] = u[d];
        q[5 + Dk + d] = 1.0 / u[d];
        C = C + (kNegHalfLog2Pi - std::log(u[d]));
      }
      o += 3 + D;
    } else if (ck == MCG_MIX_SHIFT_UNIFORM) {
      for (int d = 0; d < D; ++d) {
        if (!(u[D + d] > u[d])) return mcg::set_error(ctx, MCG_EINVAL, "MIXTURE: SHIFT_UNIFORM needs a < b");
        q[5 + d] = u[d];
        q[5 + Dk + d] = u[D + d];
        q[5 + 2 * Dk + d] = u[D + d] - u[d];
        C = C - std::log(u[D + d] - u[d]);
      }
      o += 3 + 2 * D;
    } else if (ck == MCG_MIX_WRAP_UNIFORM) {
      for (int j = 0; j < 3; ++j)
        for (int d = 0; d < D; ++d) q[5 + j * Dk + d] = u[j * D + d];
      o += 3 + 3 * D;
    } else {
      o += 3;
    }
    q[4] = C;
  }
  // The pick (mcmc.ml:168-173) walks u down the normalised weights, u - p_1 - p_2 ...; when the
  // rounded weights leave u past the last one the reference raises Failure (:173).  Every step of
  // the walk is monotone in u, so that can happen for some draw iff it happens for the largest
  // draw u53 can make, 1 - 2^-53: such weights are refused here, with the reference's message,
  // instead of failing (or, in a kernel, silently picking a component) at some later step.
  double u = 1.0 - 0x1p-53;
  bool picked = false;
  for (int c = 0; c < nc && !picked; ++c) {
    const double pc = dev[1 + c * stride];
    if (u < pc) picked = true;
    else u = u - pc;
  }
  if (!picked)
    return mcg::set_error(ctx, MCG_EFAIL, "combine_jump_proposals: internal error: no jump proposal to select "
                          "(mcmc.ml:173): the normalised weights sum below the largest uniform draw");
  return MCG_OK;
}

extern "C" {

int mcg_abi_version(void) { return MCG_ABI_VERSION; }
const char* mcg_device_arch(void) { return "gfx950"; }

const char* mcg_last_error(const mcg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int mcg_ctx_create(mcg_ctx** out, const mcg_opts* opts) {
  if (!out) return MCG_EINVAL;
  *out = nullptr;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0) return MCG_EDEVICE;
  mcg_opts o{};
  if (opts) o = *opts;
  if (o.device < 0 || o.device >= ndev) return MCG_EINVAL;
  if (o.lanes_per_chain != 0 && o.lanes_per_chain != 1 && o.lanes_per_chain != 2 &&
      o.lanes_per_chain != 4 && o.lanes_per_chain != 8)
    return MCG_EINVAL;
  mcg_ctx* ctx = new mcg_ctx();
  ctx->opts = o;
  if (hipSetDevice(o.device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) {
    delete ctx;
    return MCG_EDEVICE;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, o.device) == hipSuccess) {
    ctx->arch = prop.gcnArchName;
    ctx->num_cus = prop.multiProcessorCount;
  }
  *out = ctx;
  return MCG_OK;
}

void mcg_ctx_destroy(mcg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->opts.device);
  (void)hipStreamSynchronize(ctx->stream);
  timing_harvest(ctx);
  mcg_free_nested_bufs(ctx->nested_bufs);
  ctx->nested_bufs = nullptr;
  for (hipEvent_t e : ctx->ev_free) (void)hipEventDestroy(e);
  (void)hipEventDestroy(ctx->ev0);
  (void)hipEventDestroy(ctx->ev1);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

}  // extern "C"

namespace mcg {

// device layout of a likelihood descriptor (the layouts mcg_mh_kernel.h eval_lik reads)
int pack_likelihood(mcg_ctx* ctx, int32_t kind, int D, const double* params, size_t n,
                    std::vector<double>& dev, int32_t* is_cauchy_out, int64_t* data_n_out) {
  int32_t is_cauchy = 0;
  int64_t data_n = 0;
  dev.clear();
  switch (kind) {
    case MCG_LIK_FLAT:
      if (D < 1) return set_error(ctx, MCG_EINVAL, "FLAT: ndim >= 1");
      dev.push_back(0.0);
      break;
    case MCG_LIK_DIAG_GAUSS: {
      if (D < 1 || n != (size_t)(2 * D) || !params)
        return set_error(ctx, MCG_EINVAL, "DIAG_GAUSS: params = mu[D], sigma[D]");
      // [mu/sigma[D], 1/sigma[D], C = sum_d (-1/2 log 2pi - log sigma_d)]   (stats.ml:98-108)
      double C = 0.0;
      dev.resize(2 * D + 1);
      for (int d = 0; d < D; ++d) {
        if (!(params[D + d] > 0.0)) return set_error(ctx, MCG_EINVAL, "DIAG_GAUSS: sigma > 0");
        dev[D + d] = 1.0 / params[D + d];
        dev[d] = params[d] * dev[D + d];
        C = C + (kNegHalfLog2Pi - std::log(params[D + d]));
      }
      dev[2 * D] = C;
      break;
    }
    case MCG_LIK_GAUSS_SHELL: {
      if (D < 1 || n != (size_t)(D + 2) || !params || !(params[D + 1] > 0.0))
        return set_error(ctx, MCG_EINVAL, "GAUSS_SHELL: params = c[D], r, w (w > 0)");
      dev.assign(params, params + D);
      dev.push_back(params[D]);
      dev.push_back(1.0 / params[D + 1]);
      dev.push_back(kNegHalfLog2Pi - std::log(params[D + 1]));
      break;
    }
    case MCG_LIK_FULLCOV_GAUSS: {
      if (D < 1 || n != (size_t)(D + D * D) || !params)
        return set_error(ctx, MCG_EINVAL, "FULLCOV_GAUSS: params = mu[D], U[D*D]");
      const double* U = params + D;
      double C = 0.0;
      for (int i = 0; i < D; ++i) {
        if (!(U[i * D + i] > 0.0)) return set_error(ctx, MCG_EINVAL, "FULLCOV_GAUSS: U_ii > 0");
        C = C + (std::log(U[i * D + i]) + kNegHalfLog2Pi);
      }
      dev.assign(params, params + D);
      dev.push_back(C);
      dev.insert(dev.end(), U, U + (size_t)D * D);
      break;
    }
    case MCG_LIK_GAUSS_MIX: {
      // m, then per component mu[D], sigma[D] -> per component the DIAG block [mu/sigma[D],
      // 1/sigma[D], C_i] (stride 2D + 1); the component count rides in data_n
      if (D < 1 || !params || n < 1) return set_error(ctx, MCG_EINVAL, "GAUSS_MIX: params = m, (mu[D], sigma[D]) x m");
      const int m = (int)params[0];
      if (!(m >= 1 && m <= MCG_LIK_MIX_MAX) || (double)m != params[0] || n != 1 + (size_t)m * 2 * D)
        return set_error(ctx, MCG_EINVAL, "GAUSS_MIX: params = m (1 <= m <= %d), (mu[D], sigma[D]) x m", MCG_LIK_MIX_MAX);
      dev.assign((size_t)m * (2 * D + 1), 0.0);
      for (int c = 0; c < m; ++c) {
        const double* mu = params + 1 + (size_t)c * 2 * D;
        const double* sg = mu + D;
        double* o = &dev[(size_t)c * (2 * D + 1)];
        double C = 0.0;
        for (int d = 0; d < D; ++d) {
          if (!(sg[d] > 0.0)) return set_error(ctx, MCG_EINVAL, "GAUSS_MIX: sigma > 0");
          o[D + d] = 1.0 / sg[d];
          o[d] = mu[d] * o[D + d];
          C = C + (kNegHalfLog2Pi - std::log(sg[d]));
        }
        o[2 * D] = C;
      }
      data_n = m;
      break;
    }
    case MCG_LIK_GAUSS_DATA:
    case MCG_LIK_CAUCHY_DATA: {
      if (!params || n < 2) return set_error(ctx, MCG_EINVAL, "DATA: params = nd, data[nsamp*nd]");
      int nd = (int)params[0];
      if (nd < 1 || D != 2 * nd || (n - 1) % (size_t)nd != 0)
        return set_error(ctx, MCG_EINVAL, "DATA: ndim must be 2*nd and data a multiple of nd");
      data_n = (int64_t)((n - 1) / nd);
      dev.assign(params + 1, params + n);
      is_cauchy = kind == MCG_LIK_CAUCHY_DATA;
      break;
    }
    default:
      return set_error(ctx, MCG_EINVAL, "unknown likelihood kind %d", kind);
  }
  if (is_cauchy_out) *is_cauchy_out = is_cauchy;
  if (data_n_out) *data_n_out = data_n;
  return MCG_OK;
}

int pad_width(int32_t lik_kind, int D) {
  // the widths gen_instances.py compiles for every likelihood / proposal pair that pads
  static const int kSep[] = {1, 2, 3, 4, 5, 6, 7, 8, 12, 16, 24, 32, 48, 64};
  static const int kFull[] = {1, 2, 3, 4, 5, 6, 7, 8, 16, 32, 48, 64};
  auto first_ge = [D](const int* w, int n) {
    for (int i = 0; i < n; ++i)
      if (w[i] >= D) return w[i];
    return D;
  };
  switch (lik_kind) {
    case MCG_LIK_FLAT:
    case MCG_LIK_DIAG_GAUSS:
    case MCG_LIK_GAUSS_SHELL:
    case MCG_LIK_GAUSS_MIX: return first_ge(kSep, (int)(sizeof kSep / sizeof kSep[0]));
    case MCG_LIK_FULLCOV_GAUSS: return first_ge(kFull, (int)(sizeof kFull / sizeof kFull[0]));
    default: return D;                        // DATA kinds: (mu, sigma) halves, no padding
  }
}

std::vector<double> pad_lik(int32_t kind, int D, int DM, const std::vector<double>& v) {
  if (D == DM) return v;
  std::vector<double> o;
  switch (kind) {
    case MCG_LIK_DIAG_GAUSS:              // mu/s[D], 1/s[D], C
      o.assign(2 * (size_t)DM + 1, 0.0);
      for (int d = 0; d < D; ++d) { o[d] = v[d]; o[DM + d] = v[D + d]; }
      o[2 * DM] = v[2 * D];
      break;
    case MCG_LIK_GAUSS_MIX: {             // per component mu/s[D], 1/s[D], C_i
      const size_t m = v.size() / (2 * (size_t)D + 1);
      o.assign(m * (2 * (size_t)DM + 1), 0.0);
      for (size_t c = 0; c < m; ++c) {
        const double* src = &v[c * (2 * D + 1)];
        double* dst = &o[c * (2 * DM + 1)];
        for (int d = 0; d < D; ++d) { dst[d] = src[d]; dst[DM + d] = src[D + d]; }
        dst[2 * DM] = src[2 * D];
      }
      break;
    }
    case MCG_LIK_GAUSS_SHELL:             // c[D], R, iw, C
      o.assign((size_t)DM + 3, 0.0);
      for (int d = 0; d < D; ++d) o[d] = v[d];
      o[DM] = v[D]; o[DM + 1] = v[D + 1]; o[DM + 2] = v[D + 2];
      break;
    case MCG_LIK_FULLCOV_GAUSS:           // mu[D], C, U[D*D]
      o.assign((size_t)DM + 1 + (size_t)DM * DM, 0.0);
      for (int d = 0; d < D; ++d) o[d] = v[d];
      o[DM] = v[D];
      for (int i = 0; i < D; ++i)
        for (int j = 0; j < D; ++j) o[DM + 1 + (size_t)i * DM + j] = v[D + 1 + (size_t)i * D + j];
      break;
    default:                              // FLAT
      o.assign(1, 0.0);
  }
  return o;
}

std::vector<double> pad_prior(int D, int DM, const std::vector<double>& v, double pad_draw_lo, double pad_draw_hi) {
  if (D == DM) return v;
  std::vector<double> o(4 * (size_t)DM + 1);
  for (int d = 0; d < DM; ++d) {
    const bool in = d < D;
    o[d] = in ? v[d] : -HUGE_VAL;
    o[DM + d] = in ? v[D + d] : HUGE_VAL;
    o[2 * DM + 1 + d] = in ? v[2 * D + 1 + d] : pad_draw_lo;
    o[3 * DM + 1 + d] = in ? v[3 * D + 1 + d] : pad_draw_hi;
  }
  o[2 * DM] = v[2 * D];
  return o;
}

std::vector<double> pad_gauss_prior(int D, int DM, const std::vector<double>& v) {
  if (D == DM) return v;
  std::vector<double> o(4 * (size_t)DM + 1, 0.0);
  for (int d = 0; d < D; ++d) {
    o[d] = v[d];
    o[DM + d] = v[D + d];
    o[2 * DM + 1 + d] = v[2 * D + 1 + d];
    o[3 * DM + 1 + d] = v[3 * D + 1 + d];
  }
  o[2 * DM] = v[2 * D];
  return o;
}

std::vector<double> pad_rows(const double* rows, int64_t n, int D, int DM) {
  std::vector<double> o((size_t)n * DM, 0.0);
  for (int64_t i = 0; i < n; ++i) std::copy(rows + i * D, rows + (i + 1) * D, o.begin() + i * DM);
  return o;
}

}  // namespace mcg

extern "C" {

int mcg_set_likelihood(mcg_ctx* ctx, int32_t kind, int32_t ndim, const double* params, size_t n) {
  if (!ctx) return MCG_EINVAL;
  if (int qrc = quiesce(ctx)) return qrc;
  std::vector<double> dev;
  const int D = ndim;
  int32_t is_cauchy = 0;
  int64_t data_n = 0;
  int prc = pack_likelihood(ctx, kind, D, params, n, dev, &is_cauchy, &data_n);
  if (prc) return prc;
  const int Dk = pad_width(kind, D);
  if (ctx->D != 0 && ctx->D != D && ctx->N > 0)
    return set_error(ctx, MCG_ESTATE, "ndim changed after mcg_init (%d -> %d): call mcg_init again", ctx->D, D);
  if (ctx->D != 0 && ctx->Dk != Dk && ctx->N > 0)
    return set_error(ctx, MCG_ESTATE,
                     "likelihood kind %d runs ndim %d at kernel width %d, the chains on the device were "
                     "initialised at width %d: call mcg_init again after changing the kind",
                     kind, D, Dk, ctx->Dk);
  dev = pad_lik(kind, D, Dk, dev);
  ctx->rj_active = false;
  const bool ndim_changed = ctx->D != D;
  // the proposal and prior descriptors are laid out at the old width: re-set them below
  const bool width_changed = ctx->Dk != Dk || ctx->D != D;
  ctx->D = D;
  ctx->Dk = Dk;
  ctx->lik_kind = kind;
  ctx->is_cauchy = is_cauchy;
  ctx->data_n = data_n;
  ctx->lik_host = dev;
  int rc = hip_check(ctx, ctx->d_lik.ensure(dev.size() * 8), "alloc likelihood");
  if (rc) return rc;
  rc = hip_check(ctx, hipMemcpy(ctx->d_lik.p, dev.data(), dev.size() * 8, hipMemcpyHostToDevice), "copy likelihood");
  if (rc) return rc;
  // the prior and proposal at the new width: the same ndim (only the padding moved) keeps the
  // caller's prior and (Gaussian, wrapping or mixture) proposal, re-laid out; a new ndim starts
  // from a flat prior and the default proposal
  const bool same_ndim = ctx->pri_host.size() > 0 && ctx->prior_raw_kind >= 0 && !ndim_changed;
  if (width_changed || ctx->pri_host.size() != (size_t)(4 * Dk + 1)) {
    if (same_ndim) {
      const std::vector<double> raw = ctx->prior_raw;
      const double z = 0.0;
      rc = mcg_set_prior(ctx, ctx->prior_raw_kind, raw.empty() ? &z : raw.data(), raw.size());
    } else {
      double z = 0.0;
      rc = mcg_set_prior(ctx, MCG_PRIOR_FLAT, &z, 0);
    }
    if (rc) return rc;
  }
  if (width_changed && same_ndim && ctx->prop_raw_kind >= 0) {
    const std::vector<double> raw = ctx->prop_raw;
    if ((rc = mcg_set_proposal(ctx, ctx->prop_raw_kind, raw.data(), raw.size()))) return rc;
  } else if (width_changed) {
    // every proposal descriptor (and a kD tree) was laid out for the old ndim -- a DE proposal
    // over samples of the old width would read past its rows: back to the default proposal, a
    // unit Gaussian step at the new width, until the caller sets one of this ndim
    ctx->kd.built = false;
    double one = 1.0;
    if ((rc = mcg_set_proposal(ctx, MCG_PROP_GAUSS, &one, 1))) return rc;
  }
  return MCG_OK;
}

}  // extern "C"

namespace mcg {

// device layout: [check_lo[D], check_hi[D], lp_in, lo[D], hi[D]]: the closed-form bounds used
// by the kernels' box test, then the caller's bounds (uniform draws of nested sampling)
int pack_prior(mcg_ctx* ctx, int32_t kind, int D, const double* params, size_t n, std::vector<double>& dev) {
  dev.assign(4 * (size_t)D + 1, 0.0);
  if (kind == MCG_PRIOR_FLAT) {
    for (int d = 0; d < D; ++d) {
      dev[d] = dev[2 * D + 1 + d] = -HUGE_VAL;
      dev[D + d] = dev[3 * D + 1 + d] = HUGE_VAL;
    }
    dev[2 * D] = 0.0;
  } else if (kind == MCG_PRIOR_BOX || kind == MCG_PRIOR_OPEN_BOX) {
    if (!params || n != (size_t)(2 * D + 1))
      return set_error(ctx, MCG_EINVAL, "BOX: params = lo[D], hi[D], lp_in");
    std::copy(params, params + n, dev.begin());
    std::copy(params, params + 2 * D, dev.begin() + 2 * D + 1);
    if (kind == MCG_PRIOR_OPEN_BOX)            // lo < x < hi  <=>  nextup(lo) <= x <= nextdown(hi)
      for (int d = 0; d < D; ++d) {
        dev[d] = std::nextafter(params[d], HUGE_VAL);
        dev[D + d] = std::nextafter(params[D + d], -HUGE_VAL);
      }
  } else if (kind == MCG_PRIOR_DIAG_GAUSS) {
    // [mu/sigma[D], 1/sigma[D], C, mu[D], sigma[D]]: the DIAG_GAUSS likelihood's canonical
    // constants (the kernels evaluate lp with that same code), then the caller's mu and sigma
    // for the prior draws of nested sampling (Stats.draw_gaussian, stats.ml:113-124)
    if (!params || n != (size_t)(2 * D))
      return set_error(ctx, MCG_EINVAL, "DIAG_GAUSS prior: params = mu[D], sigma[D]");
    double C = 0.0;
    for (int d = 0; d < D; ++d) {
      if (!(params[D + d] > 0.0) || !std::isfinite(params[D + d]) || !std::isfinite(params[d]))
        return set_error(ctx, MCG_EINVAL, "DIAG_GAUSS prior: finite mu, 0 < sigma < inf");
      dev[D + d] = 1.0 / params[D + d];
      dev[d] = params[d] * dev[D + d];
      C = C + (kNegHalfLog2Pi - std::log(params[D + d]));
      dev[2 * D + 1 + d] = params[d];
      dev[3 * D + 1 + d] = params[D + d];
    }
    dev[2 * D] = C;
  } else {
    return set_error(ctx, MCG_EINVAL, "unknown prior kind %d", kind);
  }
  return MCG_OK;
}

}  // namespace mcg

extern "C" {

int mcg_set_prior(mcg_ctx* ctx, int32_t kind, const double* params, size_t n) {
  if (!ctx) return MCG_EINVAL;
  if (int qrc = quiesce(ctx)) return qrc;
  int D = ctx->D;
  if (D < 1) return set_error(ctx, MCG_ESTATE, "set the likelihood (ndim) first");
  std::vector<double> dev;
  int prc = pack_prior(ctx, kind, D, params, n, dev);
  if (prc) return prc;
  // padded dims: unbounded in the box test, drawn at 0 by nested sampling's prior draws; a
  // Gaussian prior's pad dims have zero constants (each adds +0.0 to its canonical accumulator,
  // as the DIAG_GAUSS likelihood's pad dims do) and are drawn as 0 + 0 z
  if (kind == MCG_PRIOR_DIAG_GAUSS) dev = pad_gauss_prior(D, ctx->Dk, dev);
  else dev = pad_prior(D, ctx->Dk, dev, 0.0, 0.0);
  ctx->prior_kind = kind;
  ctx->prior_raw_kind = kind;
  ctx->prior_raw.assign(params ? params : dev.data(), params ? params + n : dev.data());
  ctx->pri_host = dev;
  int rc = hip_check(ctx, ctx->d_pri.ensure(dev.size() * 8), "alloc prior");
  if (rc) return rc;
  return hip_check(ctx, hipMemcpy(ctx->d_pri.p, dev.data(), dev.size() * 8, hipMemcpyHostToDevice), "copy prior");
}

int mcg_set_proposal(mcg_ctx* ctx, int32_t kind, const double* params, size_t n) {
  if (!ctx) return MCG_EINVAL;
  if (int qrc = quiesce(ctx)) return qrc;
  int D = ctx->D;
  if (D < 1) return set_error(ctx, MCG_ESTATE, "set the likelihood (ndim) first");
  const int Dk = ctx->Dk;
  std::vector<double> dev;
  if (kind == MCG_PROP_GAUSS) {
    if (!params || (n != 1 && n != (size_t)D)) return set_error(ctx, MCG_EINVAL, "GAUSS: s[1] or s[D]");
    dev.assign(Dk, 0.0);                       // padded dims: step 0 (they stay at 0)
    for (int d = 0; d < D; ++d) dev[d] = params[n == 1 ? 0 : d];
  } else if (kind == MCG_PROP_WRAP_UNIFORM) {
    if (!params || n != (size_t)(3 * D)) return set_error(ctx, MCG_EINVAL, "WRAP_UNIFORM: lo[D], hi[D], dx[D]");
    // padded dims: the interval [0, 0) with dx 0 wraps 0 onto itself
    dev.assign(3 * (size_t)Dk, 0.0);
    for (int d = 0; d < D; ++d) {
      dev[d] = params[d];
      dev[Dk + d] = params[D + d];
      dev[2 * Dk + d] = params[2 * D + d];
    }
  } else if (kind == MCG_PROP_KD_INTERP) {
    if (!ctx->kd.built) return set_error(ctx, MCG_ESTATE, "call mcg_set_kd_proposal first");
    dev.push_back(0.0);
  } else if (kind == MCG_PROP_MIXTURE) {
    int rc = pack_mixture(ctx, params, n, dev);
    if (rc) return rc;
  } else if (kind == MCG_PROP_DE) {
    if (ctx->de_M < 2 || ctx->de_D != D)
      return set_error(ctx, MCG_ESTATE, "DE: call mcg_set_de_proposal (>= 2 samples of ndim) first");
    if (!params || n != 1 || !(params[0] >= 0.0 && params[0] <= 1.0))
      return set_error(ctx, MCG_EINVAL, "DE: params = mode_hopping_frac in [0, 1]");
    // [mode_hopping_frac, sigma = 2.38 / sqrt(2 ndim)] (mcmc.ml:212, glibc sqrt)
    dev = {params[0], 2.38 / std::sqrt(2.0 * (double)D)};
  } else {
    return set_error(ctx, MCG_EINVAL, "unsupported proposal kind %d for MH", kind);
  }
  ctx->prop_kind = kind;
  ctx->prop_host = dev;
  // (re-laid out at another kernel width from these; DE and kD need their samples / tree)
  const bool relayable = kind == MCG_PROP_GAUSS || kind == MCG_PROP_WRAP_UNIFORM ||
                         (kind == MCG_PROP_MIXTURE && !ctx->kd.built);
  ctx->prop_raw_kind = relayable ? kind : -1;
  if (relayable) ctx->prop_raw.assign(params, params + n);
  int rc = hip_check(ctx, ctx->d_prop.ensure(dev.size() * 8), "alloc proposal");
  if (rc) return rc;
  return hip_check(ctx, hipMemcpy(ctx->d_prop.p, dev.data(), dev.size() * 8, hipMemcpyHostToDevice), "copy proposal");
}

int mcg_set_kd_proposal(mcg_ctx* ctx, const double* pts, int64_t M, const double* low,
                        const double* high) {
  if (!ctx || !pts || !low || !high) return MCG_EINVAL;
  if (int qrc = quiesce(ctx)) return qrc;
  int D = ctx->D;
  if (D < 1) return set_error(ctx, MCG_ESTATE, "set the likelihood (ndim) first");
  if (M < 1) return set_error(ctx, MCG_EINVAL, "Interpolate_pdf.make: no points");
  // an ndim without a kD kernel of its own runs zero-padded at the model's width Dk (kd_build
  // pads the device boxes); the kD kernels are compiled at widths 1-8, 12 and 16 on every
  // likelihood kind, and 24 / 32 on the lane-split ones
  const int Dk = ctx->Dk;
  bool have = false;
  for (int P : {1, 2, 4, 8}) have = have || find_mh_kernel(Dk, P, ctx->lik_kind, MCG_PROP_KD_INTERP) != nullptr;
  if (!have)
    return set_error(ctx, MCG_EINVAL, "KD_INTERP: no compiled kD kernel for ndim %d (width %d) likelihood=%d",
                     D, Dk, ctx->lik_kind);
  int rc = kd_build(ctx, pts, M, D, low, high, nullptr, Dk);
  if (rc) return rc;
  double z = 0.0;
  return mcg_set_proposal(ctx, MCG_PROP_KD_INTERP, &z, 1);
}

int mcg_set_de_proposal(mcg_ctx* ctx, const double* samples, int64_t M, double mode_hopping_frac) {
  if (!ctx || !samples) return MCG_EINVAL;
  if (int qrc = quiesce(ctx)) return qrc;
  const int D = ctx->D;
  if (D < 1) return set_error(ctx, MCG_ESTATE, "set the likelihood (ndim) first");
  // pick_samples needs a j != i (mcmc.ml:202 loops forever on one sample)
  if (M < 2) return set_error(ctx, MCG_EINVAL, "differential_evolution_proposal: need >= 2 samples");
  if (M > (int64_t)0xFFFFFFFF) return set_error(ctx, MCG_EINVAL, "differential_evolution_proposal: too many samples");
  int rc;
  const int Dk = ctx->Dk;
  // rows at the kernel width (padded dims 0: the DE step y_j - x_i is 0 there)
  std::vector<double> padded;
  const double* rows = samples;
  if (Dk != D) {
    padded = pad_rows(samples, M, D, Dk);
    rows = padded.data();
  }
  if ((rc = hip_check(ctx, ctx->d_de_pts.ensure((size_t)M * Dk * 8), "alloc DE samples"))) return rc;
  if ((rc = hip_check(ctx, hipMemcpy(ctx->d_de_pts.p, rows, (size_t)M * Dk * 8, hipMemcpyHostToDevice), "copy DE samples"))) return rc;
  ctx->de_M = M;
  ctx->de_D = D;
  return mcg_set_proposal(ctx, MCG_PROP_DE, &mode_hopping_frac, 1);
}

int mcg_init(mcg_ctx* ctx, int64_t nchains, const double* x_soa, const double* ll,
             const double* lp) {
  if (!ctx || nchains < 1 || !x_soa) return MCG_EINVAL;
  if (ctx->D < 1) return set_error(ctx, MCG_ESTATE, "set the likelihood first");
  if (nchains > (int64_t)0x7FFFFFFF) return set_error(ctx, MCG_EINVAL, "too many chains");
  (void)hipSetDevice(ctx->opts.device);
  const int D = ctx->D, Dk = ctx->Dk;
  const size_t N = (size_t)nchains;
  int rc;
  // the uploads below are blocking copies on the null stream, which does not order against the
  // context's non-blocking stream: let every kernel in flight finish first
  if ((rc = quiesce(ctx))) return rc;
  // Mcmc's counters are global until reset_counters (mcmc.ml:27-35): fold this set of chains'
  // tallies into the context totals before the per-chain device counters restart
  if ((rc = mcg::fold_counters(ctx))) return rc;
  if ((rc = hip_check(ctx, ctx->d_x.ensure(N * Dk * 8), "alloc x"))) return rc;
  if ((rc = hip_check(ctx, ctx->d_ll.ensure(N * 8), "alloc ll"))) return rc;
  if ((rc = hip_check(ctx, ctx->d_lp.ensure(N * 8), "alloc lp"))) return rc;
  if ((rc = hip_check(ctx, ctx->d_nacc.ensure(N * 8), "alloc counters"))) return rc;
  // zero the (possibly new) counters before anything else can fail: mcg_get_counters reads
  // them with the old N if a later copy errors out
  if ((rc = hip_check(ctx, hipMemset(ctx->d_nacc.p, 0, N * 8), "zero counters"))) return rc;
  // [D][N] is the leading block of the [Dk][N] state; the padded rows are 0
  if ((rc = hip_check(ctx, hipMemcpy(ctx->d_x.p, x_soa, N * D * 8, hipMemcpyHostToDevice), "copy x"))) return rc;
  if (Dk > D && (rc = hip_check(ctx, hipMemset((double*)ctx->d_x.p + N * D, 0, N * (Dk - D) * 8), "zero pad rows"))) return rc;
  ctx->N = nchains;
  // steps_done is NOT reset: the Philox step counter runs on across inits like the reference's
  // global Random state (a re-init must not replay the previous draws); mcg_reseed restarts it
  ctx->last_nsteps = 0;
  ctx->nrec_total = 0;
  ctx->rec_stored = 0;
  if (ll && lp) {
    if ((rc = hip_check(ctx, hipMemcpy(ctx->d_ll.p, ll, N * 8, hipMemcpyHostToDevice), "copy ll"))) return rc;
    if ((rc = hip_check(ctx, hipMemcpy(ctx->d_lp.p, lp, N * 8, hipMemcpyHostToDevice), "copy lp"))) return rc;
    return MCG_OK;
  }
  eval_launch_fn fn = find_eval_kernel(Dk, ctx->lik_kind);
  if (!fn) return set_error(ctx, MCG_EINVAL, "no compiled kernel for likelihood %d at D=%d", ctx->lik_kind, D);
  MhArgs a = base_args(ctx);
  if ((rc = hip_check(ctx, fn(a, ctx->stream), "eval launch"))) return rc;
  return hip_check(ctx, hipStreamSynchronize(ctx->stream), "eval sync");
}

int mcg_get_state(mcg_ctx* ctx, double* x_soa, double* ll, double* lp) {
  if (!ctx) return MCG_EINVAL;
  if (ctx->N < 1) return set_error(ctx, MCG_ESTATE, "no chains");
  const size_t N = (size_t)ctx->N;
  int rc;
  if ((rc = hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync"))) return rc;
  // (the leading [D][N] block of the padded [Dk][N] state)
  if (x_soa && (rc = hip_check(ctx, hipMemcpy(x_soa, ctx->d_x.p, N * ctx->D * 8, hipMemcpyDeviceToHost), "copy x"))) return rc;
  if (ll && (rc = hip_check(ctx, hipMemcpy(ll, ctx->d_ll.p, N * 8, hipMemcpyDeviceToHost), "copy ll"))) return rc;
  if (lp && (rc = hip_check(ctx, hipMemcpy(lp, ctx->d_lp.p, N * 8, hipMemcpyDeviceToHost), "copy lp"))) return rc;
  return MCG_OK;
}

}  // extern "C"

namespace mcg {

MhArgs base_args(mcg_ctx* ctx) {
  MhArgs a{};
  a.x = (double*)ctx->d_x.p;
  a.ll = (double*)ctx->d_ll.p;
  a.lp = (double*)ctx->d_lp.p;
  a.nacc = (unsigned long long*)ctx->d_nacc.p;
  a.lik = (const double*)ctx->d_lik.p;
  a.pri = (const double*)ctx->d_pri.p;
  a.prop = (const double*)ctx->d_prop.p;
  a.N = ctx->N;
  a.k0 = (uint32_t)ctx->opts.seed;
  a.k1 = (uint32_t)(ctx->opts.seed >> 32);
  a.chain_offset = (uint32_t)ctx->opts.chain_offset;
  a.prior_kind = ctx->prior_kind;
  a.data_n = ctx->data_n;
  a.is_cauchy = ctx->is_cauchy;
  a.kd_nodes = (const KdNode*)ctx->kd.d_nodes.p;
  a.kd_logq = (const double*)ctx->kd.d_logq.p;
  a.kd_box = (const double*)ctx->kd.d_box.p;
  a.kd_pts = (const double*)ctx->kd.d_pts.p;
  a.kd_root = (const double*)ctx->kd.d_root.p;
  a.kd_pt_leaf = (const int32_t*)ctx->kd.d_pt_leaf.p;
  a.kd_M = ctx->kd.M;
  a.de_pts = (const double*)ctx->d_de_pts.p;
  a.de_M = ctx->de_M;
  if (ctx->rj_active) rj_args(ctx, a);
  // one proposal scale and one box for every dim (bitwise): the fused step takes them as scalars
  // (the descriptors are laid out at the kernel width Dk; with padding the dims D..Dk-1 hold 0
  // for the whole run, so a box applied to every dim must contain 0)
  const int D = ctx->Dk, Dr = ctx->D;
  const auto& sp = ctx->prop_host;
  const auto& bx = ctx->pri_host;
  // one box for every dim (bitwise), any proposal: eval_prior compares against kernel arguments
  // instead of loading 2D bounds per step
  const bool box_desc = ctx->prior_kind != MCG_PRIOR_DIAG_GAUSS;   // bx holds bounds (FLAT: +-inf)
  if (ctx->prior_kind != MCG_PRIOR_FLAT && box_desc && D >= 1 && (int)bx.size() >= 2 * D && !ctx->rj_active) {
    bool same = Dr == D || (bx[0] <= 0.0 && 0.0 <= bx[D]);
    for (int d = 1; d < Dr && same; ++d)
      same = !std::memcmp(&bx[d], &bx[0], 8) && !std::memcmp(&bx[D + d], &bx[D], 8);
    if (same) {
      a.ubox = 1;
      a.box_lo = bx[0];
      a.box_hi = bx[D];
    }
  }
  if (ctx->prop_kind == MCG_PROP_GAUSS && box_desc && D >= 1 && Dr == D && (int)sp.size() >= D &&
      (int)bx.size() >= 2 * D) {
    bool same = true;
    for (int d = 1; d < D && same; ++d)
      same = !std::memcmp(&sp[d], &sp[0], 8) && !std::memcmp(&bx[d], &bx[0], 8) &&
             !std::memcmp(&bx[D + d], &bx[D], 8);
    if (same) {
      a.uni = 1;
      a.uni_s = sp[0];
      a.uni_lo = bx[0];
      a.uni_hi = bx[D];
    }
  }
  return a;
}

// lanes per chain: enough lanes to put >= 4 waves on every SIMD, as long as the dimensions split
// evenly into 4-dim Philox blocks (separable likelihoods with a Gaussian proposal only).
int choose_lanes(mcg_ctx* ctx) {
  const int D = ctx->Dk;
  const bool separable = (ctx->lik_kind == MCG_LIK_DIAG_GAUSS || ctx->lik_kind == MCG_LIK_GAUSS_SHELL ||
                          ctx->lik_kind == MCG_LIK_FLAT) && ctx->prop_kind == MCG_PROP_GAUSS;
  const char* env = std::getenv("MCG_LANES_PER_CHAIN");
  int want = ctx->opts.lanes_per_chain;
  if (env && *env) want = std::atoi(env);
  // full covariance, Gaussian proposal, D in {16,32,48,64}: the matrix-core kernel (4 lanes/chain)
  // (its step tests a box prior only: a Gaussian prior runs the one-lane kernel)
  const bool fullcov_mfma = ctx->lik_kind == MCG_LIK_FULLCOV_GAUSS && ctx->prop_kind == MCG_PROP_GAUSS &&
                            ctx->prior_kind != MCG_PRIOR_DIAG_GAUSS &&
                            find_mh_kernel(D, 4, ctx->lik_kind, ctx->prop_kind) != nullptr;
  // the kD independence proposal with a separable likelihood: its draw splits over lanes too
  const bool kd_split = ctx->prop_kind == MCG_PROP_KD_INTERP &&
                        (ctx->lik_kind == MCG_LIK_DIAG_GAUSS || ctx->lik_kind == MCG_LIK_GAUSS_SHELL ||
                         ctx->lik_kind == MCG_LIK_FLAT);
  // the wrapping-uniform and DE proposals on a lane-split likelihood: wide chains split so a lane
  // holds at most 16 dims (a one-lane D 48 / 64 kernel spills 0.2-1.7 KB a lane)
  const bool wide_split = (ctx->prop_kind == MCG_PROP_WRAP_UNIFORM || ctx->prop_kind == MCG_PROP_DE) &&
                          (ctx->lik_kind == MCG_LIK_DIAG_GAUSS || ctx->lik_kind == MCG_LIK_GAUSS_SHELL ||
                           ctx->lik_kind == MCG_LIK_FLAT || ctx->lik_kind == MCG_LIK_GAUSS_MIX);
  // (the kD draw also splits two dims per lane when D = 2P: mcg_mh_kernel.h Layout W = 2)
  auto splits = [&](int P) {
    return (D % (4 * P) == 0 || (kd_split && D == 2 * P)) && find_mh_kernel(D, P, ctx->lik_kind, ctx->prop_kind);
  };
  if (want > 0) {
    if (want == 1) return 1;
    if ((separable || fullcov_mfma || kd_split || wide_split) && splits(want)) return want;
    return 1;
  }
  if (fullcov_mfma) return 4;
  if (kd_split && D > 16) {
    // kD at the wide widths (24, 32): split so a lane holds at most 16 dims, more for occupancy
    int best = 0;
    const int64_t lanes_target = (int64_t)std::max(ctx->num_cus, 1) * 4 * 4 * 64;
    for (int P : {1, 2, 4}) {
      if (D > 16 * P || !splits(P)) continue;
      if (best && ctx->N * best >= lanes_target) break;
      best = P;
    }
    return best ? best : 1;
  }
  if (wide_split) {
    for (int P : {1, 2, 4})
      if (D <= 16 * P && (P == 1 || splits(P))) return P;
    return 1;
  }
  if (!separable && !kd_split) return 1;
  const int64_t lanes_target = (int64_t)std::max(ctx->num_cus, 1) * 4 * 4 * 64;  // 4 waves/SIMD
  int best = 1;
  for (int P : {2, 4, 8}) {
    if (ctx->N * best >= lanes_target) break;
    if ((P < 8 || kd_split) && splits(P)) best = P;
  }
  return best;
}

}  // namespace mcg

extern "C" {

uint64_t mcg_state_token(const mcg_ctx* ctx) { return ctx ? ctx->state_token : 0; }

int mcg_run(mcg_ctx* ctx, const mcg_run_opts* o) {
  if (ctx) ++ctx->state_token;
  if (!ctx || !o) return MCG_EINVAL;
  if (ctx->N < 1) return set_error(ctx, MCG_ESTATE, "mcg_run before mcg_init");
  if (o->nskip < 1 || o->n_rec < 0 || o->nbin < 0) return set_error(ctx, MCG_EINVAL, "nbin >= 0, nskip >= 1, n_rec >= 0");
  if (o->append && ctx->nrec_total == 0 && o->accumulate)
    return set_error(ctx, MCG_ESTATE, "append needs a previous run with records");
  (void)hipSetDevice(ctx->opts.device);
  const int D = ctx->Dk;                   // the kernel width (the state's rows, padded)
  const int64_t N = ctx->N;
  if (!ctx->rj_active && ctx->prop_kind == MCG_PROP_DE && ctx->de_D != ctx->D)
    return set_error(ctx, MCG_ESTATE, "DE proposal samples have ndim %d, the model %d", ctx->de_D, ctx->D);
  const int P = ctx->rj_active ? 1 : choose_lanes(ctx);
  mh_launch_fn fn = ctx->rj_active ? find_rj_kernel(D) : find_mh_kernel(D, P, ctx->lik_kind, ctx->prop_kind);
  if (!fn) {
    if (D != ctx->D)
      return set_error(ctx, MCG_EINVAL, "no compiled MH kernel for ndim %d (padded to %d) likelihood=%d proposal=%d",
                       ctx->D, D, ctx->lik_kind, ctx->prop_kind);
    return set_error(ctx, MCG_EINVAL, "no compiled MH kernel for D=%d likelihood=%d proposal=%d", D, ctx->lik_kind, ctx->prop_kind);
  }
  ctx->lanes = P;
  // mcmc_array schedule: records at run-local step counts s_r = nbin + r*nskip (r < n_rec);
  // append mode records at nskip, 2 nskip, ... (no initial record).
  const bool append = o->append != 0;
  const int64_t nbin_eff = append ? o->nskip : o->nbin;
  const int64_t n_rec = o->n_rec;
  const int64_t nsteps = n_rec > 0 ? nbin_eff + (n_rec - 1) * o->nskip : o->nbin;
  const int64_t rec_base = append ? ctx->nrec_total : 0;
  int rc;
  // buffers
  const size_t Nz = (size_t)N;
  if (o->record_x && n_rec > 0) {
    if ((rc = hip_check(ctx, ctx->d_rec_x.ensure((size_t)n_rec * D * Nz * 8), "alloc rec_x"))) return rc;
  }
  if (o->record_llp && n_rec > 0) {
    if ((rc = hip_check(ctx, ctx->d_rec_ll.ensure((size_t)n_rec * Nz * 8), "alloc rec_ll"))) return rc;
    if ((rc = hip_check(ctx, ctx->d_rec_lp.ensure((size_t)n_rec * Nz * 8), "alloc rec_lp"))) return rc;
  }
  const int64_t row_bytes = ((N + 63) / 64) * 8;
  if (o->record_accept && nsteps > 0) {
    if ((rc = hip_check(ctx, ctx->d_bits.ensure((size_t)nsteps * row_bytes), "alloc accept bits"))) return rc;
    if ((rc = hip_check(ctx, hipMemsetAsync(ctx->d_bits.p, 0, (size_t)nsteps * row_bytes, ctx->stream), "zero bits"))) return rc;
  }
  if (ctx->rj_active) {
    if (o->record_llp && n_rec > 0 &&
        (rc = hip_check(ctx, ctx->d_rec_tag.ensure((size_t)n_rec * Nz), "alloc rec tags"))) return rc;
    if (o->accumulate && !append &&
        (rc = hip_check(ctx, hipMemsetAsync(ctx->d_rj_nb.p, 0, Nz * 8, ctx->stream), "zero rj counts"))) return rc;
  } else if (o->accumulate) {
    if ((rc = hip_check(ctx, ctx->d_mean.ensure(Nz * D * 8), "alloc mean"))) return rc;
    if ((rc = hip_check(ctx, ctx->d_m2.ensure(Nz * D * 8), "alloc m2"))) return rc;
    if ((rc = hip_check(ctx, ctx->d_hm_m.ensure(8 * Nz * 8), "alloc hm"))) return rc;
    if ((rc = hip_check(ctx, ctx->d_hm_s.ensure(8 * Nz * 8), "alloc hm"))) return rc;
    if (!append) {
      if ((rc = hip_check(ctx, hipMemsetAsync(ctx->d_mean.p, 0, Nz * D * 8, ctx->stream), "zero"))) return rc;
      if ((rc = hip_check(ctx, hipMemsetAsync(ctx->d_m2.p, 0, Nz * D * 8, ctx->stream), "zero"))) return rc;
      // harmonic-mean class partials: s == 0 marks an empty class
      if ((rc = hip_check(ctx, hipMemsetAsync(ctx->d_hm_s.p, 0, 8 * Nz * 8, ctx->stream), "zero"))) return rc;
    }
  }
  MhArgs a = base_args(ctx);
  a.mean = (double*)ctx->d_mean.p;
  a.m2 = (double*)ctx->d_m2.p;
  a.hm_m = (double*)ctx->d_hm_m.p;
  a.hm_s = (double*)ctx->d_hm_s.p;
  a.rec_x = (double*)ctx->d_rec_x.p;
  a.rec_ll = (double*)ctx->d_rec_ll.p;
  a.rec_lp = (double*)ctx->d_rec_lp.p;
  a.bits = (uint8_t*)ctx->d_bits.p;
  a.bits_row_bytes = row_bytes;
  a.nskip = o->nskip;
  a.rec_base = rec_base;
  a.rec_end = rec_base + n_rec;
  // Welford weights 1/(R+1) of the records (IEEE division on the host, so the kernel needs no
  // per-step division): one device table inv[R] for every absolute record index R, grown rarely.
  // (A per-run upload put a copy between consecutive MH kernels: two engine hand-offs per run.)
  {
    const int64_t need = rec_base + std::max<int64_t>(n_rec, 1) + 1;   // + the prefetch of record rec_end
    if (need > ctx->inv_cap) {
      const int64_t cap = std::max<int64_t>(need, std::max<int64_t>(2 * ctx->inv_cap, (int64_t)1 << 20));
      std::vector<double> ih((size_t)cap);
      for (int64_t q = 0; q < cap; ++q) ih[(size_t)q] = 1.0 / (double)(q + 1);
      // the running kernels may read the old table: let them finish before it is replaced
      if ((rc = hip_check(ctx, hipStreamSynchronize(ctx->stream), "inv sync"))) return rc;
      if ((rc = hip_check(ctx, ctx->d_invtab.ensure(cap * 8), "alloc inv"))) return rc;
      if ((rc = hip_check(ctx, hipMemcpy(ctx->d_invtab.p, ih.data(), cap * 8, hipMemcpyHostToDevice), "copy inv"))) return rc;
      ctx->inv_cap = cap;
    }
    a.inv_n = (const double*)ctx->d_invtab.p;
    a.next_r0 = 0;
  }
  int64_t spl = ctx->opts.steps_per_launch;
  if (const char* env = std::getenv("MCG_STEPS_PER_LAUNCH")) spl = std::atoll(env);
  if (spl <= 0) spl = std::max<int64_t>(1, std::min<int64_t>(4096, ((int64_t)1 << 26) / N));
  const int64_t nthreads = N * P;
  int64_t t0 = 0;
  bool first = true;
  do {
    const int64_t n = std::min<int64_t>(spl, nsteps - t0);
    a.t0 = t0;
    a.nsteps = n;
    a.step_base = ctx->steps_done + (uint64_t)t0;
    a.flags = (o->record_x ? RUNF_RECORD_X : 0) | (o->record_llp ? RUNF_RECORD_LLP : 0) |
              (o->record_accept ? RUNF_RECORD_ACCEPT : 0) | (o->accumulate ? RUNF_ACCUMULATE : 0);
    // first record strictly after step count t0 (the initial state is record 0 when nbin = 0)
    int64_t r_first;
    if (!append && first && nbin_eff == 0 && n_rec > 0) {
      a.flags |= RUNF_RECORD_INITIAL;
      r_first = 0;
    } else {
      r_first = (t0 < nbin_eff) ? 0 : (t0 - nbin_eff) / o->nskip + 1;
    }
    a.next_r = rec_base + r_first;
    a.next_rec = nbin_eff + r_first * o->nskip;
    if (a.flags & RUNF_RECORD_INITIAL) a.next_rec = nbin_eff + (r_first + 1) * o->nskip;
    if (n_rec == 0 || !(o->record_x || o->record_llp || o->accumulate)) a.rec_end = a.next_r;  // nothing to record
    if (n > 0 || (a.flags & RUNF_RECORD_INITIAL)) {
      hipEvent_t e0 = nullptr, e1 = nullptr;
      if (ctx->timing) timing_begin(ctx, &e0, &e1);
      if ((rc = hip_check(ctx, fn(a, nthreads, ctx->stream), "MH launch"))) return rc;
      if (ctx->timing) timing_end(ctx, e0, e1, 0);
    }
    t0 += n;
    first = false;
  } while (t0 < nsteps);
  ctx->steps_done += (uint64_t)nsteps;
  ctx->nsteps_total += nsteps;
  ctx->last_nsteps = nsteps;
  ctx->last_record_accept = o->record_accept != 0;
  if (o->accumulate) ctx->nrec_total = rec_base + n_rec;
  ctx->rec_stored = n_rec;
  ctx->rec_x_valid = o->record_x != 0;
  ctx->rec_llp_valid = o->record_llp != 0;
  return MCG_OK;
}

int64_t mcg_last_run_steps(const mcg_ctx* ctx) { return ctx ? ctx->last_nsteps : -1; }
int mcg_last_run_lanes(const mcg_ctx* ctx) { return ctx ? ctx->lanes : -1; }

int mcg_get_records(mcg_ctx* ctx, double* rec_x, double* rec_ll, double* rec_lp,
                    uint64_t* accept_bits) {
  if (!ctx) return MCG_EINVAL;
  int rc;
  if ((rc = hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync"))) return rc;
  const size_t N = (size_t)ctx->N, R = (size_t)ctx->rec_stored;
  if (rec_x) {
    if (!ctx->rec_x_valid) return set_error(ctx, MCG_ESTATE, "last run did not record x");
    if (ctx->Dk == ctx->D) {
      if ((rc = hip_check(ctx, hipMemcpy(rec_x, ctx->d_rec_x.p, R * ctx->D * N * 8, hipMemcpyDeviceToHost), "copy rec_x"))) return rc;
    } else if (R > 0) {
      // record r is [Dk][N] on the device: its leading [D][N] block
      if ((rc = hip_check(ctx, hipMemcpy2D(rec_x, (size_t)ctx->D * N * 8, ctx->d_rec_x.p, (size_t)ctx->Dk * N * 8,
                                           (size_t)ctx->D * N * 8, R, hipMemcpyDeviceToHost), "copy rec_x"))) return rc;
    }
  }
  if (rec_ll || rec_lp) {
    if (!ctx->rec_llp_valid) return set_error(ctx, MCG_ESTATE, "last run did not record ll/lp");
    if (rec_ll && (rc = hip_check(ctx, hipMemcpy(rec_ll, ctx->d_rec_ll.p, R * N * 8, hipMemcpyDeviceToHost), "copy rec_ll"))) return rc;
    if (rec_lp && (rc = hip_check(ctx, hipMemcpy(rec_lp, ctx->d_rec_lp.p, R * N * 8, hipMemcpyDeviceToHost), "copy rec_lp"))) return rc;
  }
  if (accept_bits) {
    if (!ctx->last_record_accept) return set_error(ctx, MCG_ESTATE, "last run did not record the accept bitmap");
    const size_t bytes = (size_t)ctx->last_nsteps * ((N + 63) / 64) * 8;
    if (bytes && (rc = hip_check(ctx, hipMemcpy(accept_bits, ctx->d_bits.p, bytes, hipMemcpyDeviceToHost), "copy bits"))) return rc;
  }
  return MCG_OK;
}

int mcg_get_counters(mcg_ctx* ctx, uint64_t* naccept, uint64_t* nreject) {
  if (!ctx) return MCG_EINVAL;
  if (ctx->N < 1) {
    if (naccept) *naccept = ctx->acc_base;
    if (nreject) *nreject = ctx->rej_base;
    return MCG_OK;
  }
  std::vector<uint64_t> h((size_t)ctx->N);
  int rc;
  if ((rc = hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync"))) return rc;
  if ((rc = hip_check(ctx, hipMemcpy(h.data(), ctx->d_nacc.p, h.size() * 8, hipMemcpyDeviceToHost), "copy counters"))) return rc;
  uint64_t s = 0;
  for (uint64_t v : h) s += v;
  const uint64_t total = (uint64_t)ctx->nsteps_total * (uint64_t)ctx->N;
  if (naccept) *naccept = ctx->acc_base + s;
  if (nreject) *nreject = ctx->rej_base + (total - s);
  return MCG_OK;
}

int mcg_reset_counters(mcg_ctx* ctx) {
  if (!ctx) return MCG_EINVAL;
  ++ctx->state_token;                 // the counters changed: a sampler's cached count is stale
  ctx->nsteps_total = 0;
  ctx->acc_base = ctx->rej_base = 0;
  if (ctx->N < 1) return MCG_OK;
  return hip_check(ctx, hipMemsetAsync(ctx->d_nacc.p, 0, (size_t)ctx->N * 8, ctx->stream), "reset counters");
}

int64_t mcg_num_tiles(const mcg_ctx* ctx) { return ctx ? (ctx->N + 255) / 256 : -1; }

int mcg_tile_stats_device(mcg_ctx* ctx, void** dev_ptr, int64_t* ntiles) {
  if (!ctx) return MCG_EINVAL;
  if (ctx->nrec_total < 1) return set_error(ctx, MCG_ESTATE, "no accumulated records");
  const int D = ctx->D;
  const int64_t nt = (ctx->N + 255) / 256;
  int rc;
  if ((rc = hip_check(ctx, ctx->d_tiles.ensure((size_t)nt * (2 * D + 3) * 8), "alloc tiles"))) return rc;
  TileArgs t{};
  t.mean = (const double*)ctx->d_mean.p;
  t.m2 = (const double*)ctx->d_m2.p;
  t.hm_m = (const double*)ctx->d_hm_m.p;
  t.hm_s = (const double*)ctx->d_hm_s.p;
  t.tiles = (double*)ctx->d_tiles.p;
  t.N = ctx->N;
  t.nrec = ctx->nrec_total;
  t.D = D;
  if ((rc = hip_check(ctx, launch_tile_stats(t, ctx->stream), "tile launch"))) return rc;
  if (dev_ptr) *dev_ptr = ctx->d_tiles.p;
  if (ntiles) *ntiles = nt;
  return MCG_OK;
}

int mcg_tile_stats_into(mcg_ctx* ctx, double* dev_tiles) {
  if (!ctx || !dev_tiles) return MCG_EINVAL;
  if (ctx->nrec_total < 1) return set_error(ctx, MCG_ESTATE, "no accumulated records");
  (void)hipSetDevice(ctx->opts.device);
  TileArgs t{};
  t.mean = (const double*)ctx->d_mean.p;
  t.m2 = (const double*)ctx->d_m2.p;
  t.hm_m = (const double*)ctx->d_hm_m.p;
  t.hm_s = (const double*)ctx->d_hm_s.p;
  t.tiles = dev_tiles;
  t.N = ctx->N;
  t.nrec = ctx->nrec_total;
  t.D = ctx->D;
  int rc;
  if ((rc = hip_check(ctx, launch_tile_stats(t, ctx->stream), "tile launch"))) return rc;
  return hip_check(ctx, hipStreamSynchronize(ctx->stream), "tile sync");
}

int mcg_tile_stats(mcg_ctx* ctx, double* tiles) {
  if (!ctx || !tiles) return MCG_EINVAL;
  int64_t nt = 0;
  int rc = mcg_tile_stats_device(ctx, nullptr, &nt);
  if (rc) return rc;
  if ((rc = hip_check(ctx, hipStreamSynchronize(ctx->stream), "tile sync"))) return rc;
  return hip_check(ctx, hipMemcpy(tiles, ctx->d_tiles.p, (size_t)nt * (2 * ctx->D + 3) * 8, hipMemcpyDeviceToHost), "copy tiles");
}

// Fold tiles in global order (the same Chan / log-space combine as the device tree), then
// Stats.multi_mean / multi_std (stats.ml:58-87) and log Z_HM = log n - logsumexp(-ll).
int mcg_combine_tiles(int32_t D, int64_t ntiles, const double* tiles, double* mean, double* sd,
                      double* log_z_hm) {
  if (D < 1 || ntiles < 1 || !tiles) return MCG_EINVAL;
  const int W = 2 * D + 3;
  std::vector<double> acc(W, 0.0);
  acc[2 * D + 1] = -HUGE_VAL;
  for (int64_t t = 0; t < ntiles; ++t) {
    const double* b = tiles + t * W;
    const double na = acc[0], nb = b[0];
    if (nb == 0.0) continue;
    if (na == 0.0) {
      std::copy(b, b + W, acc.begin());
      continue;
    }
    const double n = na + nb, fb = nb / n, fab = (na * nb) / n;
    for (int d = 0; d < D; ++d) {
      const double delta = b[1 + d] - acc[1 + d];
      acc[1 + d] = acc[1 + d] + delta * fb;
      acc[1 + D + d] = (acc[1 + D + d] + b[1 + D + d]) + (delta * delta) * fab;
    }
    const double ma = acc[2 * D + 1], sa = acc[2 * D + 2], mb = b[2 * D + 1], sb = b[2 * D + 2];
    const double mm = ma > mb ? ma : mb;
    acc[2 * D + 1] = mm;
    acc[2 * D + 2] = sa * host_pexp(ma - mm) + sb * host_pexp(mb - mm);
    acc[0] = n;
  }
  const double n = acc[0];
  for (int d = 0; d < D; ++d) {
    if (mean) mean[d] = acc[1 + d];
    if (sd) sd[d] = std::sqrt(acc[1 + D + d] / (n - 1.0));
  }
  if (log_z_hm) *log_z_hm = std::log(n) - (acc[2 * D + 1] + std::log(acc[2 * D + 2]));
  return MCG_OK;
}

int mcg_stats(mcg_ctx* ctx, double* mean, double* sd, double* log_z_hm) {
  if (!ctx) return MCG_EINVAL;
  const int64_t nt = mcg_num_tiles(ctx);
  std::vector<double> tiles((size_t)nt * (2 * ctx->D + 3));
  int rc = mcg_tile_stats(ctx, tiles.data());
  if (rc) return rc;
  return mcg_combine_tiles(ctx->D, nt, tiles.data(), mean, sd, log_z_hm);
}

double mcg_log_total_error_estimate(double log_ev, double log_dev, int64_t nlive) {
  // nested.ml:148-150
  const double lre2 = -std::log((double)nlive);
  double a = 2.0 * log_dev, b = lre2 + 2.0 * log_ev;
  if (a == -HUGE_VAL && b == -HUGE_VAL) return -HUGE_VAL;
  if (b > a) std::swap(a, b);
  return 0.5 * (a + std::log1p(std::exp(b - a)));
}

int mcg_posterior_samples(mcg_ctx* ctx, const double* log_wts, int64_t npts, int64_t n, int64_t* idx) {
  if (!ctx || !log_wts || npts < 1 || n < 0 || (n > 0 && !idx)) return MCG_EINVAL;
  if (n > ((int64_t)1 << 40)) return set_error(ctx, MCG_EINVAL, "posterior_samples: n too large");
  (void)hipSetDevice(ctx->opts.device);
  int rc;
  if ((rc = quiesce(ctx))) return rc;
  // summed_weights (nested.ml:170-173): sequential, glibc exp, as the reference
  std::vector<double> sums((size_t)npts);
  sums[0] = std::exp(log_wts[0]);
  for (int64_t i = 1; i < npts; ++i) sums[(size_t)i] = std::exp(log_wts[i]) + sums[(size_t)i - 1];
  DevBuf d_sums, d_idx;
  if ((rc = hip_check(ctx, d_sums.ensure((size_t)npts * 8), "alloc sums"))) return rc;
  if ((rc = hip_check(ctx, d_idx.ensure((size_t)std::max<int64_t>(n, 1) * 8), "alloc idx"))) return rc;
  if ((rc = hip_check(ctx, hipMemcpy(d_sums.p, sums.data(), (size_t)npts * 8, hipMemcpyHostToDevice), "copy sums"))) return rc;
  const uint32_t call = ctx->post_calls++;
  if ((rc = hip_check(ctx, launch_posterior_draw((const double*)d_sums.p, npts, n, (uint32_t)ctx->opts.seed,
                                                 (uint32_t)(ctx->opts.seed >> 32), call, (int64_t*)d_idx.p,
                                                 ctx->stream), "posterior launch"))) return rc;
  if ((rc = hip_check(ctx, hipStreamSynchronize(ctx->stream), "posterior sync"))) return rc;
  if (n > 0 && (rc = hip_check(ctx, hipMemcpy(idx, d_idx.p, (size_t)n * 8, hipMemcpyDeviceToHost), "copy idx"))) return rc;
  return MCG_OK;
}

int mcg_set_timing(mcg_ctx* ctx, int32_t enabled) {
  if (!ctx) return MCG_EINVAL;
  timing_harvest(ctx);
  ctx->timing = enabled != 0;
  ctx->t_mh = mcg_kernel_timing{};
  ctx->t_mh_steps = 0;
  return MCG_OK;
}

int mcg_get_kernel_timing(mcg_ctx* ctx, const char* kernel, mcg_kernel_timing* out) {
  if (!ctx || !out) return MCG_EINVAL;
  std::string k = kernel ? kernel : "mh";
  timing_harvest(ctx);
  if (k == "mh") {
    *out = ctx->t_mh;
    return MCG_OK;
  }
  if (k == "nested_walk") {
    *out = ctx->t_walk;
    return MCG_OK;
  }
  return set_error(ctx, MCG_EINVAL, "unknown kernel '%s'", k.c_str());
}

int mcg_reseed(mcg_ctx* ctx, uint64_t seed) {
  if (!ctx) return MCG_EINVAL;
  if (int rc = quiesce(ctx)) return rc;
  ctx->opts.seed = seed;
  ctx->steps_done = 0;
  ctx->post_calls = 0;
  return MCG_OK;
}

uint64_t mcg_rng_step(const mcg_ctx* ctx) { return ctx ? ctx->steps_done : 0; }

int mcg_sync(mcg_ctx* ctx) {
  if (!ctx) return MCG_EINVAL;
  return hip_check(ctx, hipStreamSynchronize(ctx->stream), "sync");
}

}  // extern "C"
