// mcg_nested.cpp -- host driver of Nested.nested_evidence (nested.ml:122-146) on the GPU.
//
// One generation = walk (k constrained DE-MCMC walkers, one lane each) -> retire (k lowest to the
// dead buffer, new points into their slots) -> estimate (running evidence + log volume) -> sort
// the k new keys -> merge them into the n-k survivors (+ stop test).  All of it is enqueued
// asynchronously in batches of generations; the device-side stop flag turns the kernels of any
// generation after the stopping one into no-ops, so the host only synchronises once per batch.
// evidence_error_and_weights (nested.ml:81-120) runs once on the host over the final points.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <utility>
#include <vector>

#include "mcg_nested_kernel.h"
#include "mcg_runtime.h"

using namespace mcg;

namespace {

struct KeyBuf {
  DevBuf ll, tie, slot;
  hipError_t ensure(int64_t n) {
    hipError_t e;
    if ((e = ll.ensure(n * 8)) != hipSuccess) return e;
    if ((e = tie.ensure(n * 8)) != hipSuccess) return e;
    return slot.ensure(n * 4);
  }
  double* l() { return (double*)ll.p; }
  long long* t() { return (long long*)tie.p; }
  int* s() { return (int*)slot.p; }
};

struct NestedBufs {
  DevBuf x, ll, lp, nx, nll, nlp, tv, prefix, qadd, st, dead_x, dead_ll, dead_lp, runl, runj;
  KeyBuf keys[2], newk, newk_tmp;
  int64_t dead_cap = 0;
};

double lse_host(double a, double b) {            // Stats.log_sum_logs (stats.ml:240-248)
  if (a == -HUGE_VAL && b == -HUGE_VAL) return -HUGE_VAL;
  if (b > a) std::swap(a, b);
  return a + std::log1p(std::exp(b - a));
}

// nested.ml:81-120; dead point i was retired with n - (i mod k) live points.
// The reference is one loop of four log-sums per point: two running sums (low, high) and two
// weight updates.  The running sums fold blocks of iterations in parallel (below); each weight
// receives at most two contributions, from the neighbouring iterations, so the weights are
// computed per index in parallel by replaying exactly those contributions in loop order.
void evidence_weights(int64_t n, int64_t nlive, int64_t k, const double* ll, double* log_ev,
                      double* log_dev, double* wts) {
  const double log_half = -0.69314718055994530942;
  const int64_t ilive = n - nlive;
  std::vector<double> prefix((size_t)k + 1, 0.0);
  for (int64_t j = 0; j < k; ++j) prefix[j + 1] = prefix[j] + std::log1p(-1.0 / (double)(nlive - j));
  auto ldv_dead = [&](int64_t i) {
    if (k == 1) return std::log(1.0 / (double)nlive) + (double)i * std::log1p(-1.0 / (double)nlive);
    const int64_t j = i % k, g = i / k;
    return std::log(1.0 / (double)(nlive - j)) + ((double)g * prefix[k] + prefix[j]);
  };
  double ldv_live;
  if (k == 1) {
    ldv_live = std::log(1.0 / (double)nlive) + (double)(ilive - 1) * std::log1p(-1.0 / (double)nlive);
  } else {
    const int64_t g = ilive / k, j = ilive % k;
    ldv_live = ((double)g * prefix[k] + prefix[j]) + std::log(1.0 / (double)nlive);
  }
  // iteration i's (dl, dh): first loop i < ilive, second loop i >= ilive (nested.ml:90-113)
  auto dl = [&](int64_t i) { return i < ilive ? ldv_dead(i) + ll[i] : ldv_live + ll[i - 1]; };
  auto dh = [&](int64_t i) { return i < ilive ? ldv_dead(i) + ll[i + 1] : ldv_live + ll[i]; };
  // running sums: sequential log-sums over blocks of kEvBlock iterations (in parallel), then a
  // sequential log-sum of the block results -- the reference's fold exactly for n <= kEvBlock,
  // within rounding beyond (the oracle folds the same blocks, oracle.c or_evidence_weights)
  constexpr int64_t kEvBlock = 65536;
  const int64_t nb = (n + kEvBlock - 1) / kEvBlock;
  std::vector<double> blow((size_t)nb, -HUGE_VAL), bhigh((size_t)nb, -HUGE_VAL);
  std::vector<std::thread> tb;
  const int TB = (int)std::max<int64_t>(1, std::min<int64_t>(nb, 8));
  for (int t = 0; t < TB; ++t)
    tb.emplace_back([&, t] {
      for (int64_t b = t; b < nb; b += TB) {
        double lo = -HUGE_VAL, hi = -HUGE_VAL;
        for (int64_t i = b * kEvBlock; i < std::min(n, (b + 1) * kEvBlock); ++i) {
          lo = lse_host(lo, dl(i));
          hi = lse_host(hi, dh(i));
        }
        blow[(size_t)b] = lo;
        bhigh[(size_t)b] = hi;
      }
    });
  // weight m: first loop dh(m-1) then dl(m); second loop dh(m) then dl(m+1)
  auto weight = [&](int64_t m) {
    double w = -HUGE_VAL;
    if (m >= 1 && m - 1 < ilive) w = lse_host(w, log_half + dh(m - 1));
    if (m < ilive) w = lse_host(w, log_half + dl(m));
    if (m >= ilive) w = lse_host(w, log_half + dh(m));
    if (m + 1 >= ilive && m + 1 < n) w = lse_host(w, log_half + dl(m + 1));
    return w;
  };
  const int T = (int)std::max<unsigned>(1, std::min<unsigned>(14, std::thread::hardware_concurrency()));
  std::vector<std::thread> tw;
  for (int t = 0; t < T; ++t)
    tw.emplace_back([&, t] {
      for (int64_t m = t * n / T; m < (t + 1) * n / T; ++m) wts[m] = weight(m);
    });
  for (auto& x : tw) x.join();
  for (auto& x : tb) x.join();
  double low = -HUGE_VAL, high = -HUGE_VAL;
  for (int64_t b = 0; b < nb; ++b) {
    low = lse_host(low, blow[(size_t)b]);
    high = lse_host(high, bhigh[(size_t)b]);
  }
  *log_ev = log_half + lse_host(low, high);
  *log_dev = high + std::log1p(-std::exp(low - high));
  const double le = *log_ev;
  tw.clear();
  for (int t = 0; t < T; ++t)
    tw.emplace_back([&, t] {
      for (int64_t m = t * n / T; m < (t + 1) * n / T; ++m) wts[m] = wts[m] - le;
    });
  for (auto& x : tw) x.join();
}

}  // namespace

struct mcg_nested_bufs_holder {
  NestedBufs b;
};

extern "C" {

int mcg_nested(mcg_ctx* ctx, const mcg_nested_opts* opts, mcg_nested_result* res,
               mcg_observer_fn observer, void* user) {
  if (!ctx || !opts) return MCG_EINVAL;
  const int D = ctx->D;
  if (D < 1) return set_error(ctx, MCG_ESTATE, "set the likelihood first");
  if (ctx->prior_kind != MCG_PRIOR_BOX && ctx->prior_kind != MCG_PRIOR_OPEN_BOX)
    return set_error(ctx, MCG_EINVAL, "nested sampling needs a box prior (draw_prior = uniform in the box)");
  const int64_t n = opts->nlive > 0 ? opts->nlive : 1000;
  const int64_t k = opts->k > 0 ? opts->k : 1;
  const int64_t nmcmc = opts->nmcmc >= 0 ? opts->nmcmc : 1000;
  const double epsrel = opts->epsrel > 0 ? opts->epsrel : 0.01;
  if (n < 2 || k >= n || n > 0x7FFFFFFF) return set_error(ctx, MCG_EINVAL, "need 2 <= nlive, 1 <= k < nlive");
  const int64_t max_dead = opts->max_dead > 0 ? opts->max_dead : 1000 * n;
  nest_walk_fn walk = find_nest_walk(D, ctx->lik_kind);
  nest_init_fn init = find_nest_init(D, ctx->lik_kind);
  if (!walk || !init) return set_error(ctx, MCG_EINVAL, "no compiled nested kernel for D=%d likelihood=%d", D, ctx->lik_kind);
  (void)hipSetDevice(ctx->opts.device);
  if (!ctx->nested_bufs) ctx->nested_bufs = new mcg_nested_bufs_holder();
  NestedBufs& B = ctx->nested_bufs->b;
  hipStream_t s = ctx->stream;
  int rc;
#define HC(expr, what) \
  if ((rc = hip_check(ctx, (expr), what))) return rc;
  int64_t p2 = 1;
  while (p2 < k) p2 <<= 1;
  HC(B.x.ensure(n * D * 8), "alloc live");
  HC(B.ll.ensure(n * 8), "alloc live");
  HC(B.lp.ensure(n * 8), "alloc live");
  HC(B.keys[0].ensure(n), "alloc keys");
  HC(B.keys[1].ensure(n), "alloc keys");
  HC(B.nx.ensure(k * D * 8), "alloc new");
  HC(B.nll.ensure(k * 8), "alloc new");
  HC(B.nlp.ensure(k * 8), "alloc new");
  HC(B.newk.ensure(k), "alloc new keys");
  HC(B.newk_tmp.ensure(k), "alloc new keys");
  HC(B.runl.ensure(((k + 255) / 256) * 256 * 8), "alloc sort runs");
  HC(B.runj.ensure(((k + 255) / 256) * 256 * 4), "alloc sort runs");
  HC(B.tv.ensure(p2 * 8), "alloc tv");
  HC(B.prefix.ensure((k + 1) * 8), "alloc prefix");
  HC(B.qadd.ensure(k * 8), "alloc qadd");
  HC(B.st.ensure(sizeof(NestDevState)), "alloc state");
  // host constants: volume prefix sums and the per-retirement log dv term of nested.ml:140
  const bool quirk = (ctx->opts.flags & MCG_FLAG_NESTED_FIXED_STOP) == 0;
  std::vector<double> prefix((size_t)k + 1, 0.0), qadd((size_t)k);
  for (int64_t j = 0; j < k; ++j) {
    prefix[j + 1] = prefix[j] + std::log1p(-1.0 / (double)(n - j));
    qadd[j] = quirk ? 1.0 / (double)(n - j) : std::log(1.0 / (double)(n - j));
  }
  HC(hipMemcpyAsync(B.prefix.p, prefix.data(), (k + 1) * 8, hipMemcpyHostToDevice, s), "copy prefix");
  HC(hipMemcpyAsync(B.qadd.p, qadd.data(), k * 8, hipMemcpyHostToDevice, s), "copy qadd");
  NestDevState st0{0.0, -HUGE_VAL, 0, 0, 0};
  HC(hipMemcpyAsync(B.st.p, &st0, sizeof st0, hipMemcpyHostToDevice, s), "copy state");

  NestArgs a{};
  a.m = base_args(ctx);
  a.x = (double*)B.x.p;
  a.ll = (double*)B.ll.p;
  a.lp = (double*)B.lp.p;
  a.nx = (double*)B.nx.p;
  a.nll = (double*)B.nll.p;
  a.nlp = (double*)B.nlp.p;
  a.newk_ll = B.newk.l();
  a.newk_tie = B.newk.t();
  a.newk_slot = B.newk.s();
  a.tv = (double*)B.tv.p;
  a.prefix = (const double*)B.prefix.p;
  a.qadd = (const double*)B.qadd.p;
  a.st = (NestDevState*)B.st.p;
  a.n = n;
  a.k = k;
  a.nmcmc = nmcmc;
  a.tv_len = p2;
  a.mode_hop = opts->mode_hop;
  a.sigma_de = 2.38 / std::sqrt(2.0 * (double)D);     // mcmc.ml:212
  a.log_epsrel = std::log(epsrel);
  a.k0 = (uint32_t)ctx->opts.seed;
  a.k1 = (uint32_t)(ctx->opts.seed >> 32);

  // initial live set: prior draws, evaluated, stably sorted by likelihood (nested.ml:126-132)
  const bool prof = std::getenv("MCG_NESTED_PROFILE") != nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  const auto t_start = now();
  HC(init(a, B.keys[0].l(), B.keys[0].t(), B.keys[0].s(), s), "nested init");
  bool in_tmp = false;
  HC(launch_sort_keys(B.keys[0].l(), B.keys[0].t(), B.keys[0].s(), B.keys[1].l(), B.keys[1].t(),
                      B.keys[1].s(), n, &in_tmp, s, nullptr), "sort live keys");
  const int base = in_tmp ? 1 : 0;                   // generation g reads keys[(base + g) % 2]

  int64_t gen = 0, reported = 0;
  int64_t batch = 4;
  NestDevState st{};
  std::vector<double> hx, hll, hlp;
  for (;;) {
    const int64_t remaining = max_dead / k - gen;
    if (remaining <= 0) break;
    const int64_t G = std::min(batch, remaining);
    const int64_t need = (gen + G) * k;
    if (need > B.dead_cap) {
      const int64_t cap = std::max<int64_t>(need, std::max<int64_t>(2 * B.dead_cap, 16 * n));
      DevBuf nxb, nlb, npb;
      HC(nxb.ensure(cap * D * 8), "alloc dead");
      HC(nlb.ensure(cap * 8), "alloc dead");
      HC(npb.ensure(cap * 8), "alloc dead");
      const int64_t used = gen * k;
      if (used > 0) {
        HC(hipMemcpyAsync(nxb.p, B.dead_x.p, used * D * 8, hipMemcpyDeviceToDevice, s), "grow dead");
        HC(hipMemcpyAsync(nlb.p, B.dead_ll.p, used * 8, hipMemcpyDeviceToDevice, s), "grow dead");
        HC(hipMemcpyAsync(npb.p, B.dead_lp.p, used * 8, hipMemcpyDeviceToDevice, s), "grow dead");
      }
      HC(hipStreamSynchronize(s), "grow dead");
      std::swap(B.dead_x.p, nxb.p); std::swap(B.dead_x.bytes, nxb.bytes);
      std::swap(B.dead_ll.p, nlb.p); std::swap(B.dead_ll.bytes, nlb.bytes);
      std::swap(B.dead_lp.p, npb.p); std::swap(B.dead_lp.bytes, npb.bytes);
      B.dead_cap = cap;
    }
    a.dead_x = (double*)B.dead_x.p;
    a.dead_ll = (double*)B.dead_ll.p;
    a.dead_lp = (double*)B.dead_lp.p;
    for (int64_t g = gen; g < gen + G; ++g) {
      KeyBuf& cur = B.keys[(base + g) % 2];
      KeyBuf& nxt = B.keys[(base + g + 1) % 2];
      a.key_ll = cur.l();
      a.key_tie = cur.t();
      a.key_slot = cur.s();
      a.mrep = g * k;
      hipEvent_t e0 = nullptr, e1 = nullptr;
      if (ctx->timing) timing_begin(ctx, &e0, &e1);
      HC(walk(a, s), "nested walk");
      if (ctx->timing) timing_end(ctx, e0, e1, 1);
      HC(launch_retire(a, D, s), "nested retire");
      HC(launch_estimate(a, s), "nested estimate");
      bool nk_tmp = false;
      if (k <= 4096) {
        // run-sorted (ll, j) scratch of ceil(k/256)*256 entries
        HC(launch_sort_new_small(a, (double*)B.runl.p, (int*)B.runj.p, B.newk_tmp.l(), B.newk_tmp.t(),
                                 B.newk_tmp.s(), s), "sort new keys");
        nk_tmp = true;
      } else {
        HC(launch_sort_keys(B.newk.l(), B.newk.t(), B.newk.s(), B.newk_tmp.l(), B.newk_tmp.t(),
                            B.newk_tmp.s(), k, &nk_tmp, s, a.st), "sort new keys");
      }
      KeyBuf& nk = nk_tmp ? B.newk_tmp : B.newk;
      HC(launch_merge_new(a, nxt.l(), nxt.t(), nxt.s(), nk.l(), nk.t(), nk.s(), s), "merge keys");
    }
    gen += G;
    HC(hipMemcpyAsync(&st, B.st.p, sizeof st, hipMemcpyDeviceToHost, s), "read state");
    HC(hipStreamSynchronize(s), "nested sync");
    const int64_t ndead = st.gen_done * k;
    if (observer && ndead > reported) {
      const int64_t m = ndead - reported;
      hx.resize(m * D); hll.resize(m); hlp.resize(m);
      HC(hipMemcpy(hx.data(), (double*)B.dead_x.p + reported * D, m * D * 8, hipMemcpyDeviceToHost), "observer copy");
      HC(hipMemcpy(hll.data(), (double*)B.dead_ll.p + reported, m * 8, hipMemcpyDeviceToHost), "observer copy");
      HC(hipMemcpy(hlp.data(), (double*)B.dead_lp.p + reported, m * 8, hipMemcpyDeviceToHost), "observer copy");
      observer(user, hx.data(), hll.data(), hlp.data(), m);
      reported = ndead;
    }
    if (st.error)
      return set_error(ctx, MCG_EFAIL, "Error in draw_new_live_point: new log(L) below the threshold");
    if (st.stopped) break;
    batch = std::min<int64_t>(batch * 2, 64);
  }
  const auto t_gen = now();
  // final: dead points in retirement order, then the live set ascending (nested.ml:143)
  const int64_t ndead = st.gen_done * k;
  const int64_t ntot = ndead + n;
  KeyBuf& fin = B.keys[(base + st.gen_done) % 2];
  NestedState& R = ctx->nested;
  // the dead rows stay on the device (B.dead_x) until mcg_nested_get copies them straight into
  // the caller's buffer; the host keeps ll / lp (for the weights) and the final live rows
  R.pts.assign((size_t)n * D, 0.0);
  R.ll.resize((size_t)ntot);
  R.lp.resize((size_t)ntot);
  R.wts.resize((size_t)ntot);
  if (ndead > 0) {
    HC(hipMemcpy(R.ll.data(), B.dead_ll.p, ndead * 8, hipMemcpyDeviceToHost), "copy dead");
    HC(hipMemcpy(R.lp.data(), B.dead_lp.p, ndead * 8, hipMemcpyDeviceToHost), "copy dead");
  }
  std::vector<int> slots((size_t)n);
  std::vector<double> lx((size_t)n * D), lll((size_t)n), llp((size_t)n);
  HC(hipMemcpy(slots.data(), fin.slot.p, n * 4, hipMemcpyDeviceToHost), "copy keys");
  HC(hipMemcpy(lx.data(), B.x.p, n * D * 8, hipMemcpyDeviceToHost), "copy live");
  HC(hipMemcpy(lll.data(), B.ll.p, n * 8, hipMemcpyDeviceToHost), "copy live");
  HC(hipMemcpy(llp.data(), B.lp.p, n * 8, hipMemcpyDeviceToHost), "copy live");
  for (int64_t j = 0; j < n; ++j) {
    const int sl = slots[(size_t)j];
    std::memcpy(&R.pts[(size_t)j * D], &lx[(size_t)sl * D], sizeof(double) * D);
    R.ll[(size_t)(ndead + j)] = lll[(size_t)sl];
    R.lp[(size_t)(ndead + j)] = llp[(size_t)sl];
  }
  const auto t_copy = now();
  evidence_weights(ntot, n, k, R.ll.data(), &R.log_ev, &R.log_dev, R.wts.data());
  if (prof)
    std::fprintf(stderr, "mcg_nested: generations %.1f ms, final copies %.1f ms, weights %.1f ms\n",
                 ms(t_start, t_gen), ms(t_gen, t_copy), ms(t_copy, now()));
  R.n_total = ntot;
  R.n_dead = ndead;
  R.n_gen = st.gen_done;
  R.nlive = n;
  if (res) {
    res->log_ev = R.log_ev;
    res->log_dev = R.log_dev;
    res->n_dead = ndead;
    res->n_total = ntot;
    res->n_gen = st.gen_done;
  }
#undef HC
  return MCG_OK;
}

int mcg_nested_get(mcg_ctx* ctx, double* pts, double* ll, double* lp, double* log_wts) {
  if (!ctx) return MCG_EINVAL;
  const NestedState& R = ctx->nested;
  if (R.n_total == 0) return set_error(ctx, MCG_ESTATE, "no nested run");
  if (pts) {
    const int64_t D = (int64_t)(R.pts.size() / (size_t)R.nlive);
    if (R.n_dead > 0) {
      int rc = hip_check(ctx, hipMemcpy(pts, ctx->nested_bufs->b.dead_x.p, (size_t)(R.n_dead * D) * 8,
                                        hipMemcpyDeviceToHost), "copy dead points");
      if (rc) return rc;
    }
    std::copy(R.pts.begin(), R.pts.end(), pts + R.n_dead * D);
  }
  if (ll) std::copy(R.ll.begin(), R.ll.end(), ll);
  if (lp) std::copy(R.lp.begin(), R.lp.end(), lp);
  if (log_wts) std::copy(R.wts.begin(), R.wts.end(), log_wts);
  return MCG_OK;
}

// Run merging for nested replicas (one independent run per GPU).  A run with
// constant live count n is n "threads"; merging runs adds their live counts at every likelihood
// level, so R runs of n/R points each merge into one run of n points.  The volume and trapezoid
// algebra is that of evidence_error_and_weights (nested.ml:81-120) with a per-point live count.
int mcg_nested_merge(int32_t nruns, const int64_t* n_total, const int64_t* nlive, const int64_t* k,
                     const double* ll, int64_t* order, double* log_ev, double* log_dev,
                     double* log_wts) {
  if (nruns <= 0 || !n_total || !nlive || !k || !ll || !order || !log_ev || !log_dev || !log_wts)
    return MCG_EINVAL;
  std::vector<int64_t> base((size_t)nruns + 1, 0);
  for (int r = 0; r < nruns; ++r) {
    if (nlive[r] <= 0 || k[r] <= 0 || k[r] > nlive[r] || n_total[r] < nlive[r]) return MCG_EINVAL;
    base[(size_t)r + 1] = base[(size_t)r] + n_total[r];
  }
  const int64_t n = base[(size_t)nruns];
  // live count of run r's point i
  auto count = [&](int r, int64_t i) -> int64_t {
    const int64_t ndead = n_total[r] - nlive[r];
    return i < ndead ? nlive[r] - i % k[r] : nlive[r] - (i - ndead);
  };
  for (int64_t p = 0; p < n; ++p) order[p] = p;
  // ascending ll; ties by concatenation index (= run, then position in the run)
  std::stable_sort(order, order + n, [&](int64_t a, int64_t b) { return ll[a] < ll[b]; });
  // pos[r] = first index of run r with ll >= the current level; ll is nondecreasing within a run
  std::vector<int64_t> pos((size_t)nruns, 0);
  const double log_half = -0.69314718055994530942;
  double log_x = 0.0, low = -HUGE_VAL, high = -HUGE_VAL;
  for (int64_t p = 0; p < n; ++p) log_wts[p] = -HUGE_VAL;
  for (int64_t p = 0; p < n; ++p) {
    const double L = ll[order[p]];
    int64_t np = 0;
    for (int r = 0; r < nruns; ++r) {
      int64_t& i = pos[(size_t)r];
      while (i < n_total[r] && ll[base[(size_t)r] + i] < L) ++i;
      if (i < n_total[r]) np += count(r, i);
    }
    const double log_dv = log_x + std::log(1.0 / (double)np);
    log_x += std::log1p(-1.0 / (double)np);
    const int64_t q = p + 1 < n ? p + 1 : p;
    const double dl = log_dv + L, dh = log_dv + ll[order[q]];
    low = lse_host(low, dl);
    high = lse_host(high, dh);
    log_wts[p] = lse_host(log_wts[p], log_half + dl);
    log_wts[q] = lse_host(log_wts[q], log_half + dh);
  }
  *log_ev = log_half + lse_host(low, high);
  *log_dev = high + std::log1p(-std::exp(low - high));
  for (int64_t p = 0; p < n; ++p) log_wts[p] -= *log_ev;
  return MCG_OK;
}

}  // extern "C"

void mcg_free_nested_bufs(mcg_nested_bufs_holder* h) { delete h; }
