// mcg_nested.cpp -- host driver of Nested.nested_evidence (nested.ml:122-146) on the GPU.
//
// One generation = walk (k constrained DE-MCMC walkers, one lane each) -> retire (k lowest to the
// dead buffer, new points into their slots) -> estimate (running evidence + log volume) -> sort
// the k new keys -> merge them into the n-k survivors (+ stop test).  All of it is enqueued
// asynchronously in batches of generations; the device-side stop flag turns the kernels of any
// generation after the stopping one into no-ops, so the host only synchronises once per batch.
// Batches are pipelined: while the GPU runs batch b + 1, a host worker folds batch b's dead
// points into evidence_error_and_weights (nested.ml:81-120); the live points are folded in once
// the run has stopped.
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
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
  DevBuf samp_ll, samp_tie;   // every kKeySample-th key (indices 63, 127, ...): merge search samples
  hipError_t ensure(int64_t n) {
    hipError_t e;
    if ((e = ll.ensure(n * 8)) != hipSuccess) return e;
    if ((e = tie.ensure(n * 8)) != hipSuccess) return e;
    if ((e = samp_ll.ensure((n / kKeySample + 1) * 8)) != hipSuccess) return e;
    if ((e = samp_tie.ensure((n / kKeySample + 1) * 8)) != hipSuccess) return e;
    return slot.ensure(n * 4);
  }
  double* l() { return (double*)ll.p; }
  long long* t() { return (long long*)tie.p; }
  int* s() { return (int*)slot.p; }
  double* sl() { return (double*)samp_ll.p; }
  long long* st() { return (long long*)samp_tie.p; }
};

struct NestedBufs {
  DevBuf x, ll, lp, nx, nll, nlp, tv, prefix, qadd, st, dead_x, dead_ll, dead_lp, rank, sync, trace, chk, rt_ix, rt_sc,
      fm_sync;
  KeyBuf keys[2], newk, newk_tmp;
  int64_t dead_cap = 0;
  // pinned staging of two in-flight batches' dead (ll, lp) and their completion events; coherent
  // and device-mapped: the kernels that retire points write them there directly (d_stage)
  double* h_stage[4] = {nullptr, nullptr, nullptr, nullptr};
  double* d_stage[4] = {nullptr, nullptr, nullptr, nullptr};
  int64_t h_cap = 0;
  NestDevState* h_st = nullptr;
  hipEvent_t done[2] = {nullptr, nullptr};
  // pinned chunk ring of the large device -> host copy in mcg_nested_get (copy_d2h_large)
  static constexpr int kRing = 4;
  static constexpr size_t kRingChunk = (size_t)16 << 20;
  void* h_ring[kRing] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t ev_ring[kRing] = {nullptr, nullptr, nullptr, nullptr};
  ~NestedBufs() {
    for (auto h : h_ring)
      if (h) (void)hipHostFree(h);
    for (auto e : ev_ring)
      if (e) (void)hipEventDestroy(e);
    for (auto h : h_stage)
      if (h) (void)hipHostFree(h);
    if (h_st) (void)hipHostFree(h_st);
    for (auto e : done)
      if (e) (void)hipEventDestroy(e);
  }
};

double lse_host(double a, double b) {            // Stats.log_sum_logs (stats.ml:240-248)
  if (a == -HUGE_VAL && b == -HUGE_VAL) return -HUGE_VAL;
  // one side -inf: exp(-inf) = 0 and log1p(0) = 0, so the sum is the other side + 0.0 (the
  // same bits, without the two libm calls)
  if (a == -HUGE_VAL) return b + 0.0;
  if (b == -HUGE_VAL) return a + 0.0;
  if (b > a) std::swap(a, b);
  return a + std::log1p(std::exp(b - a));
}

// nested.ml:81-120; dead point i was retired with n - (i mod k) live points.
// The reference is one loop of four log-sums per point: two running sums (low, high) and two
// weight updates.  The running sums fold blocks of kEvBlock iterations (in parallel), then fold
// the block results in order -- the reference's fold exactly for n <= kEvBlock, within rounding
// beyond (the oracle folds the same blocks, oracle.c or_evidence_weights).  Each weight receives
// at most two contributions, from the neighbouring iterations, so the weights are computed per
// index in parallel by replaying exactly those contributions in loop order.
//
// The fold is incremental: while the GPU runs a batch of generations, advance() folds every
// block and weight whose inputs are dead points already on the host; finish() does the rest
// (the live points, ldv_live) once the run has stopped.
constexpr int64_t kEvBlock = 65536;
constexpr int64_t kWeightChunk = 16384;                 // weights per fold task
constexpr double kLogHalf = -0.69314718055994530942;

template <class F>
void parallel_for(int64_t lo, int64_t hi, int threads, F f) {
  if (hi <= lo) return;
  const int64_t T = std::max<int64_t>(1, std::min<int64_t>(threads, hi - lo));
  if (T == 1) {
    for (int64_t i = lo; i < hi; ++i) f(i);
    return;
  }
  std::vector<std::thread> tw;
  for (int64_t t = 0; t < T; ++t)
    tw.emplace_back([&, t] {
      for (int64_t i = lo + t * (hi - lo) / T; i < lo + (t + 1) * (hi - lo) / T; ++i) f(i);
    });
  for (auto& x : tw) x.join();
}

// tasks [0, n) on `threads` threads, handed out one at a time (the block folds are long, the
// weight chunks short: a static split would leave threads idle behind a block)
template <class F>
void parallel_tasks(int64_t n, int threads, F f) {
  if (n <= 0) return;
  const int64_t T = std::max<int64_t>(1, std::min<int64_t>(threads, n));
  if (T == 1) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<int64_t> next{0};
  auto run = [&] {
    for (int64_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < n;) f(i);
  };
  std::vector<std::thread> tw;
  for (int64_t t = 1; t < T; ++t) tw.emplace_back(run);
  run();
  for (auto& x : tw) x.join();
}

class EvFold {
 public:
  EvFold(int64_t nlive, int64_t k) : n_(nlive), k_(k), prefix_((size_t)k + 1, 0.0), lfrac_((size_t)k) {
    for (int64_t j = 0; j < k; ++j) prefix_[j + 1] = prefix_[j] + std::log1p(-1.0 / (double)(nlive - j));
    // log(1 / (n - j)) of every retirement slot j, and the k = 1 terms of nested.ml:96, computed
    // once (the per-point log was most of the fold's time; the same values bit for bit)
    for (int64_t j = 0; j < k; ++j) lfrac_[(size_t)j] = std::log(1.0 / (double)(nlive - j));
    l1_ = std::log(1.0 / (double)nlive);
    l1p_ = std::log1p(-1.0 / (double)nlive);
    threads_ = (int)std::max<unsigned>(1, std::min<unsigned>(14, std::thread::hardware_concurrency()));
    // while the GPU runs (on the fold worker, beside the launching thread)
    const char* e = std::getenv("MCG_NESTED_FOLD_THREADS");
    stream_threads_ = std::max(1, std::min(threads_, e ? std::atoi(e) : 12));
  }

  // ll[0, avail) are dead points (avail <= ilive): fold the blocks and weights that need no
  // later point; wts must hold avail entries
  void advance(const double* ll, int64_t avail, double* wts) {
    View v{this, ll, INT64_MAX, 0.0};
    // block b is complete when its last iteration's ll[i + 1] is known: (b + 1) B < avail;
    // weight m (dead, with m + 1 dead too) needs ll[m] only: m < avail - 1.  The block folds
    // (sequential inside a block) and the weight chunks run as one task list.
    const int64_t nb = avail > 0 ? (avail - 1) / kEvBlock : 0;
    const int64_t wend = std::max<int64_t>(wdone_, avail - 1);
    fold_and_weigh(v, nb, wend, wts, stream_threads_);
    wdone_ = wend;
  }

  // all ntot points known (ilive dead ones): fold the rest, combine, normalise
  // (normalise = false leaves wts[m] = log w_m + log Z: the caller subtracts *log_ev when it
  // copies them out, the same subtraction as here)
  void finish(const double* ll, int64_t ntot, double* wts, double* log_ev, double* log_dev, bool normalise = true) {
    const int64_t ilive = ntot - n_;
    View v{this, ll, ilive, 0.0};
    v.ntot = ntot;
    // the final live points each get 1/nlive of the volume that remained before the last
    // retirement: nested.ml:104 is log_vol_fraction + log X_(ilive-1), X_(ilive-1) the product
    // of the first ilive-1 volume reductions.  For k > 1 the same X is the generation prefix
    // (not the last dead point's own element, which divides by its live count nlive - k + 1
    // and so would over-weight the live points by nlive / (nlive - k + 1))
    if (k_ == 1) {
      v.ldv_live = std::log(1.0 / (double)n_) + (double)(ilive - 1) * std::log1p(-1.0 / (double)n_);
    } else if (ilive > 0) {
      const int64_t m = ilive - 1, j = m % k_, g = m / k_;
      v.ldv_live = std::log(1.0 / (double)n_) + ((double)g * prefix_[(size_t)k_] + prefix_[(size_t)j]);
    } else {
      v.ldv_live = std::log(1.0 / (double)n_);
    }
    fold_and_weigh(v, (ntot + kEvBlock - 1) / kEvBlock, ntot, wts, threads_);
    double low = -HUGE_VAL, high = -HUGE_VAL;
    for (size_t b = 0; b < blow_.size(); ++b) {
      low = lse_host(low, blow_[b]);
      high = lse_host(high, bhigh_[b]);
    }
    *log_ev = kLogHalf + lse_host(low, high);
    *log_dev = high + std::log1p(-std::exp(low - high));
    if (!normalise) return;
    const double le = *log_ev;
    parallel_for(0, threads_, threads_, [&](int64_t t) {
      for (int64_t m = t * ntot / threads_; m < (t + 1) * ntot / threads_; ++m) wts[m] -= le;
    });
  }

 private:
  struct View {
    const EvFold* f;
    const double* ll;
    int64_t ilive;                      // INT64_MAX while streaming (every index is dead)
    double ldv_live;
    int64_t ntot = INT64_MAX;
    double ldv_dead(int64_t i) const {
      if (f->k_ == 1) return f->l1_ + (double)i * f->l1p_;
      const int64_t j = i % f->k_, g = i / f->k_;
      return f->lfrac_[(size_t)j] + ((double)g * f->prefix_[(size_t)f->k_] + f->prefix_[(size_t)j]);
    }
    // iteration i's (dl, dh): first loop i < ilive, second loop i >= ilive (nested.ml:90-113)
    double dl(int64_t i) const { return i < ilive ? ldv_dead(i) + ll[i] : ldv_live + ll[i - 1]; }
    double dh(int64_t i) const { return i < ilive ? ldv_dead(i) + ll[i + 1] : ldv_live + ll[i]; }
    // weight m: first loop dh(m-1) then dl(m); second loop dh(m) then dl(m+1)
    double weight(int64_t m) const {
      double w = -HUGE_VAL;
      if (m >= 1 && m - 1 < ilive) w = lse_host(w, kLogHalf + dh(m - 1));
      if (m < ilive) w = lse_host(w, kLogHalf + dl(m));
      if (m >= ilive) w = lse_host(w, kLogHalf + dh(m));
      if (m + 1 >= ilive && m + 1 < ntot) w = lse_host(w, kLogHalf + dl(m + 1));
      return w;
    }
  };

  // blocks [blow_.size(), nb) folded and weights [wdone_, wend) computed, as one task list
  void fold_and_weigh(const View& v, int64_t nb, int64_t wend, double* wts, int threads) {
    const int64_t b0 = (int64_t)blow_.size();
    const int64_t nbt = std::max<int64_t>(0, nb - b0);
    if (nbt) {
      blow_.resize((size_t)nb, -HUGE_VAL);
      bhigh_.resize((size_t)nb, -HUGE_VAL);
    }
    const int64_t end = std::min<int64_t>(v.ntot, nb * kEvBlock);
    const int64_t w0 = wdone_, nw = std::max<int64_t>(0, wend - w0);
    const int64_t nwt = (nw + kWeightChunk - 1) / kWeightChunk;
    // a block's two running sums (low, high) are independent folds: two tasks
    parallel_tasks(2 * nbt + nwt, threads, [&](int64_t task) {
      if (task < 2 * nbt) {
        const int64_t b = b0 + task / 2;
        const int64_t i1 = std::min(end, (b + 1) * kEvBlock);
        double acc = -HUGE_VAL;
        if (task & 1) {
          for (int64_t i = b * kEvBlock; i < i1; ++i) acc = lse_host(acc, v.dh(i));
          bhigh_[(size_t)b] = acc;
        } else {
          for (int64_t i = b * kEvBlock; i < i1; ++i) acc = lse_host(acc, v.dl(i));
          blow_[(size_t)b] = acc;
        }
      } else {
        const int64_t m0 = w0 + (task - 2 * nbt) * kWeightChunk;
        const int64_t m1 = std::min(wend, m0 + kWeightChunk);
        for (int64_t m = m0; m < m1; ++m) wts[m] = v.weight(m);
      }
    });
  }

  int64_t n_, k_;
  std::vector<double> prefix_, lfrac_;
  double l1_ = 0.0, l1p_ = 0.0;
  int threads_ = 1, stream_threads_ = 1;
  std::vector<double> blow_, bhigh_;
  int64_t wdone_ = 0;
};

}  // namespace

struct mcg_nested_bufs_holder {
  NestedBufs b;
};

extern "C" {

int mcg_nested(mcg_ctx* ctx, const mcg_nested_opts* opts, mcg_nested_result* res,
               mcg_observer_fn observer, void* user) {
  if (!ctx || !opts) return MCG_EINVAL;
  ++ctx->state_token;
  // D: the kernel width of the live rows [n][D] (the caller's ndim Dr, zero-padded to a
  // compiled width; the padding is stripped from every point handed back)
  const int D = ctx->Dk, Dr = ctx->D;
  if (D < 1) return set_error(ctx, MCG_ESTATE, "set the likelihood first");
  if (ctx->rj_active) return set_error(ctx, MCG_ESTATE, "nested sampling after mcg_set_rjmcmc: set a likelihood first");
  const bool box_prior = ctx->prior_kind == MCG_PRIOR_BOX || ctx->prior_kind == MCG_PRIOR_OPEN_BOX;
  if (!box_prior && ctx->prior_kind != MCG_PRIOR_DIAG_GAUSS)
    return set_error(ctx, MCG_EINVAL, "nested sampling needs a box or DIAG_GAUSS prior (a draw_prior)");
  // the box's log density enters every walker step's MH ratio as lp_box - lp_box = +0: a finite
  // value is what makes that test always pass (mcg_nested_kernel.h, the shell walker's step)
  if (box_prior && !std::isfinite(ctx->pri_host[2 * D]))
    return set_error(ctx, MCG_EINVAL, "nested sampling needs a finite box log density");
  const int64_t n = opts->nlive > 0 ? opts->nlive : 1000;
  const int64_t k = opts->k > 0 ? opts->k : 1;
  const int64_t nmcmc = opts->nmcmc >= 0 ? opts->nmcmc : 1000;
  const double epsrel = opts->epsrel > 0 ? opts->epsrel : 0.01;
  if (n < 2 || k >= n || n > 0x7FFFFFFF) return set_error(ctx, MCG_EINVAL, "need 2 <= nlive, 1 <= k < nlive");
  // the generation's estimate tree holds 16 retirements per thread of one 1024-thread workgroup
  if (k > 16384) return set_error(ctx, MCG_EINVAL, "k (points retired per generation) must be <= 16384");
  if (nmcmc > 0x7FFFFFF0) return set_error(ctx, MCG_EINVAL, "nmcmc must be < 2^31");   // walker step counters
  const int64_t max_dead = opts->max_dead > 0 ? opts->max_dead : 1000 * n;
  nest_walk_fn walk = find_nest_walk(D, ctx->lik_kind);
  nest_init_fn init = find_nest_init(D, ctx->lik_kind);
  if (!walk || !init) return set_error(ctx, MCG_EINVAL, "no compiled nested kernel for ndim %d (width %d) likelihood=%d", Dr, D, ctx->lik_kind);
  (void)hipSetDevice(ctx->opts.device);
  // forget the previous run up front: a run that fails below must not leave mcg_nested_get
  // sizing its copies from the previous run's counts over this run's partial data
  {
    NestedState& R0 = ctx->nested;
    R0.n_total = R0.n_dead = R0.n_gen = 0;
    R0.converged = false;
  }
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
  HC(B.rank.ensure(k * 4), "alloc new-key ranks");
  HC(B.sync.ensure(2 * kSyncUse * 4), "alloc hand-off counters");
  HC(hipMemsetAsync(B.sync.p, 0, 2 * kSyncUse * 4, s), "clear hand-off counters");
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
  NestDevState st0{{0.0, 0.0}, {-HUGE_VAL, -HUGE_VAL}, 0, 0, 0, -HUGE_VAL};
  HC(hipMemcpyAsync(B.st.p, &st0, sizeof st0, hipMemcpyHostToDevice, s), "copy state");

  NestArgs a{};
  a.m = base_args(ctx);
  {
    // a box prior symmetric in every dim (closed form lo[d] == -hi[d], bitwise): the walkers
    // test it as |y| <= hi, one compare per dim
    const auto& bx = ctx->pri_host;
    bool sym = box_prior && (int64_t)bx.size() >= 2 * D;
    for (int64_t d = 0; d < D && sym; ++d) {
      const double nhi = -bx[(size_t)(D + d)];
      sym = !std::memcmp(&bx[(size_t)d], &nhi, 8);
    }
    a.sym_box = sym ? 1 : 0;
  }
  a.x = (double*)B.x.p;
  a.ll = (double*)B.ll.p;
  a.lp = (double*)B.lp.p;
  a.nx = (double*)B.nx.p;
  a.nll = (double*)B.nll.p;
  a.nlp = (double*)B.nlp.p;
  a.newk_ll = B.newk.l();
  a.newk_tie = B.newk.t();
  a.newk_slot = B.newk.s();
  a.rank = (int*)B.rank.p;
  // k <= 8192: retirement in the walk and the sort + merge in one launch, whose extra workgroup
  // folds the estimate; MCG_NESTED_MERGE2=1 keeps the counted-rank sort (k <= 4096, the estimate
  // in its extra workgroup) and the merge as two launches; beyond, the retire kernel folds it
  const bool merge2 = std::getenv("MCG_NESTED_MERGE2") != nullptr;
  const bool retire_kernel = std::getenv("MCG_NESTED_RETIRE_KERNEL") != nullptr;
  const bool fused_merge = !merge2 && !retire_kernel && k <= 8192;
  a.est_in_rank = (fused_merge || k <= 4096) ? 1 : 0;
  // MCG_NEST_LANES: lanes per walker (8 for D % 32 == 0; 4 at D = 8, 8 at D = 16: two dims per
  // lane), "wide" for that wider split, "narrow" for the one-block-per-call split
  if (const char* e = std::getenv("MCG_NEST_LANES"))
    a.lanes_hint = !std::strcmp(e, "wide") ? -1 : !std::strcmp(e, "narrow") ? -2 : std::atoi(e);
  a.fuse_retire = a.est_in_rank && !retire_kernel;
  // MCG_NESTED_FM=1 (k <= 4096 with the draw table): the merge runs in the walk's launch
  // (nest_walk_kernel's merge role, one kernel boundary a generation instead of two).  Not the
  // default: measured slower at C3
  const char* fm_env = std::getenv("MCG_NESTED_FM");
  const bool fuse_walk_merge = fused_merge && k <= 4096 && fm_env && fm_env[0] == '1';
  a.fm_sync = nullptr;
  if (fuse_walk_merge) {
    // group counters, top counter and one go flag per merge workgroup, 128 B apart, zeroed per run
    const int64_t words = (kSyncGroups + 1 + (n - k + 255) / 256 + 1) * kSyncStride;
    HC(B.fm_sync.ensure(words * 4), "alloc hand-off flags");
    HC(hipMemsetAsync(B.fm_sync.p, 0, words * 4, s), "clear hand-off flags");
    a.fm_sync = (uint32_t*)B.fm_sync.p;
  }
  // the walkers' draws of a generation in a table the previous merge fills (when it fits)
  a.rt_ix = nullptr;
  a.rt_sc = nullptr;
  // (its DE pairs are stored as row byte offsets i D 8 | j D 8 << 32, so the live set must span
  // less than 4 GiB)
  a.row_bytes = (uint32_t)(D * 8);
  if (2 * k * (nmcmc + kWalkTabPad) * 24 <= ((int64_t)512 << 20) && (uint64_t)n * (uint64_t)D * 8u < ((uint64_t)1 << 32) &&
      std::getenv("MCG_NESTED_NO_TABLE") == nullptr) {
    // two halves of nmcmc + kWalkTabPad rows; the pad rows stay zero (walk_tab_base)
    const int64_t ent = 2 * k * (nmcmc + kWalkTabPad);
    HC(B.rt_ix.ensure(ent * 8), "alloc draw table");
    HC(B.rt_sc.ensure(ent * 16), "alloc draw table");
    HC(hipMemsetAsync(B.rt_ix.p, 0, ent * 8, s), "clear draw table");
    HC(hipMemsetAsync(B.rt_sc.p, 0, ent * 16, s), "clear draw table");
    a.rt_ix = (unsigned long long*)B.rt_ix.p;
    a.rt_sc = (double2*)B.rt_sc.p;
  }
  // Split merge (MCG_NESTED_SPLIT=1, opt-in): the head of each
  // generation's merge (keys [0, k), kernel merge_head_kernel) on the critical path, its tail
  // (positions >= k) and the generation's estimate inside the next walk's launch.  Needs the draw
  // table's walk layout and the in-walk retirement.  Bit-exact, but measured slower at C3 than
  // the one-launch merge of every position (the default)
  int base_off = 0;                                  // set once the initial sort has run
  auto base_keys = [&](int64_t g) { return base_off + g; };
  const char* sp_env = std::getenv("MCG_NESTED_SPLIT");
  const bool split = fused_merge && !fuse_walk_merge && k <= kSmallSort && a.fuse_retire && a.rt_ix &&
                     sp_env && sp_env[0] == '1';
  const int32_t tail_nblk = (int32_t)((n - k + 255) / 256);
  auto set_tail = [&](int64_t gp) {                  // the tail of generation gp
    KeyBuf& in = B.keys[(base_keys(gp)) % 2];
    KeyBuf& out = B.keys[(base_keys(gp + 1)) % 2];
    KeyBuf& nk = (gp & 1) ? B.newk_tmp : B.newk;
    a.tl_nblk = tail_nblk;
    a.tl_mrep = gp * k;
    a.tl_gen1 = gp + 1;
    a.tl_key_ll = in.l();
    a.tl_key_tie = in.t();
    a.tl_key_slot = in.s();
    a.tl_newk_ll = nk.l();
    a.tl_newk_slot = nk.s();
    a.tl_out_ll = out.l();
    a.tl_out_tie = out.t();
    a.tl_out_slot = out.s();
    a.tl_samp_ll = out.sl();
    a.tl_samp_tie = out.st();
  };
  a.split = split ? 1 : 0;
  a.est_in_walk = split ? 1 : 0;
  a.sync = (uint32_t*)B.sync.p;
  a.tv = (double*)B.tv.p;
  a.prefix = (const double*)B.prefix.p;
  a.qadd = (const double*)B.qadd.p;
  a.st = (NestDevState*)B.st.p;
  a.n = n;
  a.k = k;
  a.nmcmc = nmcmc;
  a.tv_len = p2;
  a.mode_hop = opts->mode_hop;
  a.sigma_de = 2.38 / std::sqrt(2.0 * (double)Dr);    // mcmc.ml:212 (the caller's ndim)
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
  base_off = base;
  HC(launch_key_sample(B.keys[base].l(), B.keys[base].t(), n, B.keys[base].sl(), B.keys[base].st(), s, a.st),
     "sample live keys");
  HC(launch_walk_draws(a, 0, s), "first draws");

  // Batches of generations, pipelined: while the GPU runs batch b + 1, the host appends batch b's
  // dead ll / lp (copied into pinned staging behind b's kernels) and folds them into the
  // evidence sums (EvFold::advance).  The dead rows themselves stay on the device.
  NestedState& R = ctx->nested;
  R.ll.clear();
  R.lp.clear();
  R.wts.clear();
  R.taken = false;
  // (the blocks a take left for this run may still be prefaulting: joined before any of them
  // can be reallocated)
  EvFold fold(n, k);
  // generations per batch: doubling from 4 up to kMaxBatch (MCG_NESTED_MAX_BATCH)
  const char* mb_env = std::getenv("MCG_NESTED_MAX_BATCH");
  const int64_t kMaxBatch = std::max<int64_t>(4, mb_env ? std::atoll(mb_env) : 64);
  if (B.h_cap < kMaxBatch * k) {
    for (auto& h : B.h_stage) {
      if (h) (void)hipHostFree(h);
      h = nullptr;
    }
    for (int i = 0; i < 4; ++i) {
      HC(hipHostMalloc(&B.h_stage[i], (size_t)(kMaxBatch * k) * 8,
                       hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable),
         "alloc pinned staging");
      HC(hipHostGetDevicePointer((void**)&B.d_stage[i], B.h_stage[i], 0), "map pinned staging");
    }
    B.h_cap = kMaxBatch * k;
  }
  // MCG_NESTED_STAGE_COPY=1: stage each batch's dead ll / lp by two device-to-host copies behind
  // its kernels instead (the copies are blit kernels on the same queue, ~38 us each at C3)
  const bool stage_copy = std::getenv("MCG_NESTED_STAGE_COPY") != nullptr;
  // the state copies land in pinned memory too: an async copy into pageable memory would block
  // the host until the batch completes and serialise the pipeline
  if (!B.h_st) HC(hipHostMalloc((void**)&B.h_st, 2 * sizeof(NestDevState), 0), "alloc pinned state");
  NestDevState* hst = B.h_st;
  int64_t gen = 0, reported = 0, batch = 4;
  const bool check = std::getenv("MCG_NESTED_CHECK") != nullptr;
  if (check) {
    HC(B.chk.ensure(4 * 8), "alloc check");
    HC(hipMemsetAsync(B.chk.p, 0, 4 * 8, s), "clear check");
  }
#ifdef MCG_NEST_TRACE
  // phase stamps of one generation (MCG_NEST_TRACE=<generation>), printed at the end
  const char* trace_env = std::getenv("MCG_NEST_TRACE");
  const int64_t trace_gen = trace_env ? std::atoll(trace_env) : -1;
  if (trace_gen >= 0) {
    HC(B.trace.ensure(4 * 1024 * 8 * 8), "alloc trace");
    HC(hipMemsetAsync(B.trace.p, 0, 4 * 1024 * 8 * 8, s), "clear trace");
  }
#endif
  // Dead buffers replaced while batches were in flight (tagged with the sequence number of the
  // batch whose launch replaced them) are freed when the run ends, after the stream has drained.
  // Not earlier: they come from hipMalloc, and a hipFree mid-run would wait for the batches in
  // flight (undoing the refill-before-join overlap), while hipFreeAsync is specified for
  // stream-ordered pool allocations only.  The buffers double in size at each grow,
  // so the retired ones hold at most as much as the live one.
  struct RetiredBufs {
    hipStream_t s;
    std::vector<std::pair<int64_t, void*>> bufs;
    ~RetiredBufs() {
      if (bufs.empty()) return;
      (void)hipStreamSynchronize(s);
      for (auto& e : bufs) (void)hipFree(e.second);
    }
  } retired_dead{s, {}};
  int64_t batch_seq = 0;                              // batches launched so far
  int64_t slot_seq[2] = {-1, -1};                     // the batch in each slot
  // enqueue generations [gen, gen + G) and the copies of their state / dead ll, lp into slot q
  // the dead-row buffer each in-flight batch's kernels write: once the batch's done event has
  // fired it holds every row up to the batch's end (earlier rows were written there or copied in
  // by a grow copy queued ahead of the batch), while B.dead_x may already be a newer buffer whose
  // grow copy is still queued behind the other batch
  double* slot_dead_x[2] = {nullptr, nullptr};
  auto launch_batch = [&](int64_t G, int q) -> int {
    const int64_t need = (gen + G) * k;
    if (need > B.dead_cap) {
      // room for the live rows too (gathered behind the dead ones at the end)
      const int64_t cap = std::max<int64_t>(need + n, std::max<int64_t>(2 * B.dead_cap, 16 * n));
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
      // no host sync: the copies are stream-ordered behind every kernel that writes the old
      // buffers and ahead of every kernel that writes the new ones; the old buffers are freed
      // once the run has drained (retired_dead)
      std::swap(B.dead_x.p, nxb.p); std::swap(B.dead_x.bytes, nxb.bytes);
      std::swap(B.dead_ll.p, nlb.p); std::swap(B.dead_ll.bytes, nlb.bytes);
      std::swap(B.dead_lp.p, npb.p); std::swap(B.dead_lp.bytes, npb.bytes);
      for (DevBuf* o : {&nxb, &nlb, &npb}) {
        retired_dead.bufs.push_back({batch_seq, o->p});
        o->p = nullptr;
        o->bytes = 0;
      }
      B.dead_cap = cap;
    }
    a.dead_x = (double*)B.dead_x.p;
    a.dead_ll = (double*)B.dead_ll.p;
    a.dead_lp = (double*)B.dead_lp.p;
    a.h_ll = stage_copy ? nullptr : B.d_stage[2 * q];
    a.h_lp = stage_copy ? nullptr : B.d_stage[2 * q + 1];
    a.h_m0 = gen * k;
    slot_dead_x[q] = a.dead_x;
    slot_seq[q] = batch_seq++;
    for (int64_t g = gen; g < gen + G; ++g) {
      KeyBuf& cur = B.keys[(base + g) % 2];
      KeyBuf& nxt = B.keys[(base + g + 1) % 2];
      a.key_ll = cur.l();
      a.key_tie = cur.t();
      a.key_slot = cur.s();
      a.key_samp_ll = cur.sl();
      a.key_samp_tie = cur.st();
      a.out_samp_ll = nxt.sl();
      a.out_samp_tie = nxt.st();
      a.mrep = g * k;
#ifdef MCG_NEST_TRACE
      a.trace = (g == trace_gen) ? (unsigned long long*)B.trace.p : nullptr;
#endif
      hipEvent_t e0 = nullptr, e1 = nullptr;
      if (ctx->timing) timing_begin(ctx, &e0, &e1);
      a.mrg_ll = nxt.l();
      a.mrg_tie = nxt.t();
      a.mrg_slot = nxt.s();
      a.fuse_merge = (fuse_walk_merge && a.rt_ix) ? 1 : 0;
      if (split) {
        // this generation's new keys go to half g & 1 (the tail in this launch reads the other)
        KeyBuf& nk = (g & 1) ? B.newk_tmp : B.newk;
        a.newk_ll = nk.l();
        a.newk_tie = nk.t();
        a.newk_slot = nk.s();
        if (g > 0) set_tail(g - 1);
        else a.tl_nblk = 0;
      }
      HC(walk(a, s), "nested walk");
      if (ctx->timing) timing_end(ctx, e0, e1, 1);
      if (split) {
        // generation g - 1's keys are complete once this walk (its tail) has run
        if (check && g > 0) HC(launch_check_sorted(cur.l(), cur.t(), n, g - 1, (long long*)B.chk.p + 1, s), "check");
        HC(launch_merge_head(a, nxt.l(), nxt.t(), nxt.s(), s), "merge head");
        continue;
      }
      if (a.fuse_merge) {                 // merged in the walk's launch (or right after it)
        if (check) HC(launch_check_sorted(nxt.l(), nxt.t(), n, g, (long long*)B.chk.p + 1, s), "check");
        continue;
      }
      if (fused_merge) {
        // the new keys sorted and merged into the survivors in one launch (merge_fused_kernel)
        HC(launch_merge_fused(a, nxt.l(), nxt.t(), nxt.s(), s), "merge keys");
        if (check) HC(launch_check_sorted(nxt.l(), nxt.t(), n, g, (long long*)B.chk.p + 1, s), "check");
        continue;
      }
      if (!a.fuse_retire) HC(launch_retire(a, D, s), "nested retire");
      bool nk_tmp = false;
      if (k <= 4096) {
        HC(launch_sort_new_small(a, B.newk_tmp.l(), B.newk_tmp.t(), B.newk_tmp.s(), s), "sort new keys");
        nk_tmp = true;
      } else {
        HC(launch_sort_keys(B.newk.l(), B.newk.t(), B.newk.s(), B.newk_tmp.l(), B.newk_tmp.t(),
                            B.newk_tmp.s(), k, &nk_tmp, s, a.st), "sort new keys");
      }
      KeyBuf& nk = nk_tmp ? B.newk_tmp : B.newk;
      if (check) HC(launch_check_sorted(nk.l(), nk.t(), k, g, (long long*)B.chk.p, s), "check");
      HC(launch_merge_new(a, nxt.l(), nxt.t(), nxt.s(), nk.l(), nk.t(), nk.s(), s), "merge keys");
      if (check) HC(launch_check_sorted(nxt.l(), nxt.t(), n, g, (long long*)B.chk.p + 1, s), "check");
    }
    HC(hipMemcpyAsync(&hst[q], B.st.p, sizeof(NestDevState), hipMemcpyDeviceToHost, s), "read state");
    if (stage_copy) {
      HC(hipMemcpyAsync(B.h_stage[2 * q], (double*)B.dead_ll.p + gen * k, G * k * 8, hipMemcpyDeviceToHost, s),
         "stage dead ll");
      HC(hipMemcpyAsync(B.h_stage[2 * q + 1], (double*)B.dead_lp.p + gen * k, G * k * 8, hipMemcpyDeviceToHost, s),
         "stage dead lp");
    }
    HC(hipEventRecord(B.done[q], s), "record batch");
    gen += G;
    return MCG_OK;
  };
  for (auto& e : B.done)
    if (!e) HC(hipEventCreateWithFlags(&e, hipEventDisableTiming), "create event");
  int q = 0;
  double t_launch = 0, t_wait = 0, t_fold = 0, t_first = -1;
  std::thread fw;                                     // fold worker (EvFold::advance)
  struct Joiner {
    std::thread& t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } fw_guard{fw};
  int64_t G = std::min<int64_t>(batch, max_dead / k);
  if (G <= 0) return set_error(ctx, MCG_EINVAL, "max_dead below one generation");
  // Two batches in flight: while the GPU runs the batch in one slot, the other slot's batch is
  // already enqueued behind it, so the GPU does not idle while the host wakes up, reads a
  // finished batch's state and enqueues the next one.  A batch enqueued past the stop runs as
  // no-ops (every kernel tests the stop flag).
  int64_t gstart[2] = {0, 0};
  bool inflight[2] = {false, false};
  gstart[q] = gen;
  const double t_setup = ms(t_start, now());
  if ((rc = launch_batch(G, q))) return rc;
  inflight[q] = true;
  if (max_dead / k - gen > 0) {
    batch = std::min<int64_t>(batch * 2, kMaxBatch);
    gstart[q ^ 1] = gen;
    if ((rc = launch_batch(std::min(batch, max_dead / k - gen), q ^ 1))) return rc;
    inflight[q ^ 1] = true;
  }
  NestDevState st{};
  std::vector<double> hx;
  for (;;) {
    const auto tw0 = now();
    HC(hipEventSynchronize(B.done[q]), "nested sync");
    t_wait += ms(tw0, now());
    if (t_first < 0) t_first = ms(t_start, now());
    inflight[q] = false;
    st = hst[q];
    if (st.error) {
      if (inflight[q ^ 1]) (void)hipEventSynchronize(B.done[q ^ 1]);
      if (st.error == 2)                             // (MCG_NESTED_FM) a merge workgroup's bounded wait
        return set_error(ctx, MCG_EFAIL, "nested: the walk -> merge hand-off timed out (MCG_NESTED_FM)");
      return set_error(ctx, MCG_EFAIL, "Error in draw_new_live_point: new log(L) below the threshold");
    }
    auto join_fold = [&] {
      const auto tf = now();
      if (fw.joinable()) fw.join();
      t_fold += ms(tf, now());
    };
    // this batch's dead points: generations [gstart[q], st.gen_done) of the ones it launched.
    // The fold worker reads R.ll through a pointer taken when it started, so R.ll may grow under
    // it only within its capacity (the worker is joined first when it must reallocate)
    const int64_t d0 = gstart[q] * k, d1 = st.gen_done * k;
    if (d1 > d0) {
      if (R.ll.capacity() < R.ll.size() + (size_t)(d1 - d0) || R.lp.capacity() < R.lp.size() + (size_t)(d1 - d0)) {
        join_fold();
        R.join_populate();
        if (!R.ll.reserve(std::max(2 * R.ll.capacity(), R.ll.size() + (size_t)(d1 - d0) + (size_t)(kMaxBatch * k))))
          return set_error(ctx, MCG_EFAIL, "out of host memory");
      }
      if (!R.ll.append(B.h_stage[2 * q], B.h_stage[2 * q] + (d1 - d0)) ||
          !R.lp.append(B.h_stage[2 * q + 1], B.h_stage[2 * q + 1] + (d1 - d0)))
        return set_error(ctx, MCG_EFAIL, "out of host memory");
    }
    const double* done_dead_x = slot_dead_x[q];      // (before the refill below replaces it)
    const int64_t remaining = max_dead / k - gen;
    if (!st.stopped && remaining > 0) {               // the slot is free again: refill it
      batch = std::min<int64_t>(batch * 2, kMaxBatch);
      gstart[q] = gen;
      const auto tl = now();
      if ((rc = launch_batch(std::min(batch, remaining), q))) return rc;
      t_launch += ms(tl, now());
      inflight[q] = true;
    }
    const int64_t ndead = d1;
    if (observer && ndead > reported) {
      const int64_t m = ndead - reported;
      hx.resize(m * Dr);
      // the rows of this finished batch's buffer (complete up to its end: no stream wait needed)
      HC(hipMemcpy2D(hx.data(), (size_t)Dr * 8, done_dead_x + reported * D, (size_t)D * 8, (size_t)Dr * 8, m,
                     hipMemcpyDeviceToHost), "observer copy");
      observer(user, hx.data(), R.ll.data() + reported, R.lp.data() + reported, m);
      reported = ndead;
    }
    // the refill above went out before this join: the fold of the last batch never holds up the
    // GPU's next batch
    join_fold();
    if (st.stopped) {
      // a batch enqueued past the stop retires nothing; let it drain before the final copies
      if (inflight[q ^ 1]) HC(hipEventSynchronize(B.done[q ^ 1]), "nested sync");
      break;
    }
    if (!inflight[q] && !inflight[q ^ 1]) break;      // max_dead reached
    // fold what is final on the worker while this thread keeps the GPU fed
    if (R.wts.capacity() < R.ll.size()) R.join_populate();
    if (!R.wts.resize(R.ll.size())) return set_error(ctx, MCG_EFAIL, "out of host memory");
    fw = std::thread([&fold, llp = R.ll.data(), av = (int64_t)R.ll.size(), wp = R.wts.data()] {
      fold.advance(llp, av, wp);
    });
    q ^= 1;
  }
  if (split && st.gen_done > 0) {
    // the last generation's tail: run by the walk that found the stop, not at all when the run
    // ended at max_dead; idempotent, so it is always enqueued
    set_tail(st.gen_done - 1);
    HC(launch_merge_tail(a, s), "merge tail");
    if (check)
      HC(launch_check_sorted(B.keys[(base + st.gen_done) % 2].l(), B.keys[(base + st.gen_done) % 2].t(), n,
                             st.gen_done - 1, (long long*)B.chk.p + 1, s), "check");
  }
  const auto t_gen = now();
#ifdef MCG_NEST_TRACE
  if (trace_gen >= 0 && trace_gen < st.gen_done) {
    std::vector<unsigned long long> tr(4 * 1024 * 8);
    HC(hipMemcpy(tr.data(), B.trace.p, tr.size() * 8, hipMemcpyDeviceToHost), "copy trace");
    unsigned long long t0 = ~0ull;
    for (int b = 0; b < 1024; ++b)
      if (tr[(size_t)b * 8]) t0 = std::min(t0, tr[(size_t)b * 8]);
    const char* names[4] = {"walk", "retire", "rank_count", "merge_new"};
    for (int kid = 0; kid < 4; ++kid)
      for (int sl = 0; sl < 8; ++sl) {
        std::vector<double> v;
        for (int b = 0; b < 1024; ++b) {
          const unsigned long long x = tr[((size_t)kid * 1024 + b) * 8 + sl];
          if (x) v.push_back((double)(x - t0) * 0.01);          // 100 MHz -> us
        }
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        std::fprintf(stderr, "trace gen %lld %-10s slot %d: n %4zu  min %7.2f  med %7.2f  max %7.2f us\n",
                     (long long)trace_gen, names[kid], sl, v.size(), v.front(), v[v.size() / 2], v.back());
      }
  }
#endif
  if (prof)
    std::fprintf(stderr, "mcg_nested: host launch %.1f ms, wait %.1f ms, fold join %.1f ms, setup %.2f ms, first batch done at %.2f ms, "
                 "%lld generations launched for %lld run\n", t_launch, t_wait, t_fold, t_setup, t_first, (long long)gen,
                 (long long)st.gen_done);
  // final: dead points in retirement order, then the live set ascending (nested.ml:143)
  const int64_t ndead = st.gen_done * k;
  const int64_t ntot = ndead + n;
  KeyBuf& fin = B.keys[(base + st.gen_done) % 2];
  // every row stays on the device: the live rows are gathered in key order behind the dead rows
  // (B.dead_x), where mcg_nested_get copies all of them straight into the caller's buffer; the
  // host gets ll / lp (for the weights)
  if (ntot > B.dead_cap) {
    DevBuf nxb, nlb, npb;
    HC(nxb.ensure(ntot * D * 8), "alloc dead");
    HC(nlb.ensure(ntot * 8), "alloc dead");
    HC(npb.ensure(ntot * 8), "alloc dead");
    if (ndead > 0) {
      HC(hipMemcpyAsync(nxb.p, B.dead_x.p, ndead * D * 8, hipMemcpyDeviceToDevice, s), "grow dead");
      HC(hipMemcpyAsync(nlb.p, B.dead_ll.p, ndead * 8, hipMemcpyDeviceToDevice, s), "grow dead");
      HC(hipMemcpyAsync(npb.p, B.dead_lp.p, ndead * 8, hipMemcpyDeviceToDevice, s), "grow dead");
    }
    HC(hipStreamSynchronize(s), "grow dead");
    std::swap(B.dead_x.p, nxb.p); std::swap(B.dead_x.bytes, nxb.bytes);
    std::swap(B.dead_ll.p, nlb.p); std::swap(B.dead_ll.bytes, nlb.bytes);
    std::swap(B.dead_lp.p, npb.p); std::swap(B.dead_lp.bytes, npb.bytes);
    B.dead_cap = ntot;
  }
  HC(launch_gather_live((const double*)B.x.p, (const double*)B.ll.p, (const double*)B.lp.p, fin.s(), n, D,
                        (double*)B.dead_x.p + ndead * D, (double*)B.dead_ll.p + ndead,
                        (double*)B.dead_lp.p + ndead, s), "gather live");
  R.join_populate();
  if (!R.ll.resize((size_t)ntot) || !R.lp.resize((size_t)ntot) || !R.wts.resize((size_t)ntot))
    return set_error(ctx, MCG_EFAIL, "out of host memory");
  HC(hipMemcpyAsync(R.ll.data() + ndead, (double*)B.dead_ll.p + ndead, n * 8, hipMemcpyDeviceToHost, s), "copy live");
  HC(hipMemcpyAsync(R.lp.data() + ndead, (double*)B.dead_lp.p + ndead, n * 8, hipMemcpyDeviceToHost, s), "copy live");
  HC(hipStreamSynchronize(s), "copy live");
  if (std::getenv("MCG_NESTED_CHECK")) {
    // diagnostics: device-side sortedness of every generation, and the final keys against the
    // live ll they index
    long long ck[4];
    std::vector<double> kl((size_t)n);
    HC(hipMemcpy(ck, B.chk.p, sizeof ck, hipMemcpyDeviceToHost), "check");
    HC(hipMemcpy(kl.data(), fin.ll.p, n * 8, hipMemcpyDeviceToHost), "check");
    int64_t incons = 0, unsorted = 0;
    for (int64_t j = 0; j < n; ++j) {
      incons += R.ll[(size_t)(ndead + j)] != kl[(size_t)j];
      if (j && kl[(size_t)j] < kl[(size_t)j - 1]) ++unsorted;
    }
    std::fprintf(stderr, "mcg_nested check: first unsorted generation+1: new keys %lld, merged %lld; final keys "
                 "vs live ll mismatches %lld, unsorted keys %lld\n", ck[0], ck[1], (long long)incons,
                 (long long)unsorted);
  }
  const auto t_copy = now();
  // the weights' normalisation (w - log Z) happens in mcg_nested_get's copy, not in a pass here
  fold.finish(R.ll.data(), ntot, R.wts.data(), &R.log_ev, &R.log_dev, false);
  R.wts_shift = R.log_ev;
  if (prof)
    std::fprintf(stderr, "mcg_nested: generations %.1f ms, final copies %.1f ms, weights %.1f ms\n",
                 ms(t_start, t_gen), ms(t_gen, t_copy), ms(t_copy, now()));
  R.n_total = ntot;
  R.converged = st.stopped != 0;
  R.n_dead = ndead;
  R.ndim = Dr;
  R.ndim_k = D;
  R.n_gen = st.gen_done;
  R.nlive = n;
  if (res) {
    res->log_ev = R.log_ev;
    res->log_dev = R.log_dev;
    res->n_dead = ndead;
    res->n_total = ntot;
    res->n_gen = st.gen_done;
    res->converged = st.stopped ? 1 : 0;
  }
#undef HC
  return MCG_OK;
}

// Device -> pageable host copy of a large buffer (the dead rows: 457 MB at C3).  A plain pageable
// hipMemcpy stages through the driver with one host thread; here the DMA fills a ring of pinned
// chunks while host threads copy finished chunks into the destination in parallel.
static hipError_t copy_d2h_large(NestedBufs& B, void* dst, const void* src, size_t bytes, hipStream_t s) {
  constexpr int R = NestedBufs::kRing;
  constexpr size_t CH = NestedBufs::kRingChunk;
  if (bytes <= CH) return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
  for (int r = 0; r < R; ++r) {
    hipError_t e;
    if (!B.h_ring[r] && (e = hipHostMalloc(&B.h_ring[r], CH, 0)) != hipSuccess) return e;
    if (!B.ev_ring[r] && (e = hipEventCreateWithFlags(&B.ev_ring[r], hipEventDisableTiming)) != hipSuccess) return e;
  }
  {
    // the destination is usually fresh (numpy) memory: ask for transparent huge pages, so first
    // touch takes ~1/512 of the page faults (advice only; ignored where THP is off)
    const uintptr_t a0 = ((uintptr_t)dst + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
    const uintptr_t a1 = ((uintptr_t)dst + bytes) & ~(uintptr_t)((2u << 20) - 1);
    if (a1 > a0) (void)madvise((void*)a0, a1 - a0, MADV_HUGEPAGE);
  }
  const size_t nch = (bytes + CH - 1) / CH;
  auto len = [&](size_t c) { return std::min(CH, bytes - c * CH); };
  auto enqueue = [&](size_t c) -> hipError_t {
    const int r = (int)(c % R);
    hipError_t e = hipMemcpyAsync(B.h_ring[r], (const char*)src + c * CH, len(c), hipMemcpyDeviceToHost, s);
    return e == hipSuccess ? hipEventRecord(B.ev_ring[r], s) : e;
  };
  hipError_t err = hipSuccess;
  for (size_t c = 0; c < nch && c < (size_t)R && err == hipSuccess; ++c) err = enqueue(c);
  if (err != hipSuccess) return err;
  const int T = (int)std::max<unsigned>(1, std::min<unsigned>(8, std::thread::hardware_concurrency()));
  std::atomic<int64_t> ready{-1};                    // last chunk whose DMA has completed
  std::atomic<int64_t> copied{0};                    // worker slices copied
  std::atomic<bool> abort{false};
  auto slice = [&](size_t c, int w) {
    const size_t n = len(c), a = n * (size_t)w / T, b = n * (size_t)(w + 1) / T;
    std::memcpy((char*)dst + c * CH + a, (const char*)B.h_ring[c % R] + a, b - a);
  };
  std::vector<std::thread> pool;
  for (int w = 1; w < T; ++w)
    pool.emplace_back([&, w] {
      for (size_t c = 0; c < nch; ++c) {
        while (ready.load(std::memory_order_acquire) < (int64_t)c) {
          if (abort.load(std::memory_order_relaxed)) return;
          std::this_thread::yield();
        }
        slice(c, w);
        copied.fetch_add(1, std::memory_order_release);
      }
    });
  for (size_t c = 0; c < nch; ++c) {
    if ((err = hipEventSynchronize(B.ev_ring[c % R])) != hipSuccess) break;
    ready.store((int64_t)c, std::memory_order_release);
    slice(c, 0);
    while (copied.load(std::memory_order_acquire) < (int64_t)((c + 1) * (size_t)(T - 1))) std::this_thread::yield();
    if (c + R < nch && (err = enqueue(c + R)) != hipSuccess) break;
  }
  if (err != hipSuccess) abort.store(true);
  for (auto& t : pool) t.join();
  return err;
}

int mcg_nested_get(mcg_ctx* ctx, double* pts, double* ll, double* lp, double* log_wts) {
  if (!ctx) return MCG_EINVAL;
  const NestedState& R = ctx->nested;
  if (R.n_total == 0) return set_error(ctx, MCG_ESTATE, "no nested run");
  const auto t0 = std::chrono::steady_clock::now();
  if (pts) {
    NestedBufs& B = ctx->nested_bufs->b;
    int rc;
    if (R.ndim_k == R.ndim) {
      rc = hip_check(ctx, copy_d2h_large(B, pts, B.dead_x.p, (size_t)(R.n_total * R.ndim) * 8, ctx->stream),
                     "copy points");
    } else {
      // rows [n_total][ndim_k] on the device: their leading ndim columns
      rc = hip_check(ctx, hipMemcpy2D(pts, (size_t)R.ndim * 8, B.dead_x.p, (size_t)R.ndim_k * 8, (size_t)R.ndim * 8,
                                      (size_t)R.n_total, hipMemcpyDeviceToHost), "copy points");
    }
    if (rc) return rc;
  }
  const auto t1 = std::chrono::steady_clock::now();
  if (R.taken && (ll || lp || log_wts))
    return set_error(ctx, MCG_ESTATE, "the run's ll / lp / weights were handed over (mcg_nested_take)");
  {
    // the three host arrays in chunks over 8 threads (first touch of the caller's pages
    // dominates: the destinations get transparent-huge-page advice, as the point copy's)
    const size_t n = R.ll.size();
    double* dst[3] = {ll, lp, log_wts};
    const double* srcs[3] = {R.ll.data(), R.lp.data(), R.wts.data()};
    for (double* d : dst) {
      if (!d || n * 8 < (4u << 20)) continue;
      const uintptr_t a0 = ((uintptr_t)d + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
      const uintptr_t a1 = ((uintptr_t)d + n * 8) & ~(uintptr_t)((2u << 20) - 1);
      if (a1 > a0) (void)madvise((void*)a0, a1 - a0, MADV_HUGEPAGE);
    }
    constexpr int kT = 8;
    const double sh = R.wts_shift;
    auto work = [&](int t) {
      const size_t c0 = n * t / kT, c1 = n * (t + 1) / kT;
      for (int q = 0; q < 2; ++q)
        if (dst[q]) std::copy(srcs[q] + c0, srcs[q] + c1, dst[q] + c0);
      if (dst[2])                                     // log weights: normalised here (EvFold::finish)
        for (size_t i = c0; i < c1; ++i) dst[2][i] = srcs[2][i] - sh;
    };
    if (n < ((size_t)1 << 16)) {
      work(0);
      for (int t = 1; t < kT; ++t) work(t);
    } else {
      std::thread th[kT - 1];
      for (int t = 1; t < kT; ++t) th[t - 1] = std::thread(work, t);
      work(0);
      for (auto& x : th) x.join();
    }
  }
  if (std::getenv("MCG_NESTED_PROFILE"))
    std::fprintf(stderr, "mcg_nested_get: points %.1f ms, ll/lp/wts %.1f ms\n",
                 std::chrono::duration<double, std::milli>(t1 - t0).count(),
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
  return MCG_OK;
}

int mcg_nested_take(mcg_ctx* ctx, double** ll, double** lp, double** log_wts) {
  if (!ctx || !ll || !lp || !log_wts) return MCG_EINVAL;
  NestedState& R = ctx->nested;
  if (R.n_total == 0) return set_error(ctx, MCG_ESTATE, "no nested run");
  if (R.taken) return set_error(ctx, MCG_ESTATE, "the run's ll / lp / weights were already handed over");
  // the log weights normalised in place (w - log Z, as mcg_nested_get's copy does), over 8 threads
  const size_t n = R.wts.size();
  double* w = R.wts.data();
  const double sh = R.wts_shift;
  constexpr int kT = 8;
  auto work = [&](int t) {
    const size_t c0 = n * t / kT, c1 = n * (t + 1) / kT;
    for (size_t i = c0; i < c1; ++i) w[i] -= sh;
  };
  if (n < ((size_t)1 << 16)) {
    for (int t = 0; t < kT; ++t) work(t);
  } else {
    std::thread th[kT - 1];
    for (int t = 1; t < kT; ++t) th[t - 1] = std::thread(work, t);
    work(0);
    for (auto& x : th) x.join();
  }
  R.join_populate();
  *ll = R.ll.release();
  *lp = R.lp.release();
  *log_wts = R.wts.release();
  R.taken = true;
  // fresh blocks for the next run, sized like this one, prefaulted in the background (the page
  // zeroing a fresh block costs would otherwise land on the next run's host loop)
  const size_t cap = (size_t)R.n_total + (size_t)R.n_total / 8;
  if (R.ll.reserve_fresh(cap) && R.lp.reserve_fresh(cap) && R.wts.reserve_fresh(cap)) {
    double* blocks[3] = {R.ll.data(), R.lp.data(), R.wts.data()};
    const size_t bytes = R.ll.capacity() * sizeof(double);
    R.populate = std::thread([blocks, bytes] {
      for (double* b : blocks) (void)madvise(b, bytes, MADV_POPULATE_WRITE);
    });
  }
  return MCG_OK;
}

void mcg_free(void* p) { std::free(p); }

int mcg_nested_rows_into(mcg_ctx* ctx, double* dev_rows, int64_t row_stride, int32_t with_points) {
  if (!ctx || !dev_rows) return MCG_EINVAL;
  const NestedState& R = ctx->nested;
  if (R.n_total == 0 || !ctx->nested_bufs) return set_error(ctx, MCG_ESTATE, "no nested run");
  if (row_stride < (with_points ? R.ndim : 0) + 2)
    return set_error(ctx, MCG_EINVAL, "row_stride %lld < %d", (long long)row_stride, (with_points ? R.ndim : 0) + 2);
  (void)hipSetDevice(ctx->opts.device);
  NestedBufs& B = ctx->nested_bufs->b;
  int rc;
  if ((rc = hip_check(ctx, launch_nested_rows((const double*)B.dead_x.p, R.ndim_k, R.ndim, (const double*)B.dead_ll.p,
                                              (const double*)B.dead_lp.p, R.n_total, dev_rows, row_stride,
                                              with_points ? 1 : 0, ctx->stream), "rows launch")))
    return rc;
  return hip_check(ctx, hipStreamSynchronize(ctx->stream), "rows sync");
}

int mcg_evidence_weights(int64_t ntot, int64_t nlive, int64_t k, const double* ll, int64_t chunk,
                         double* log_ev, double* log_dev, double* log_wts) {
  if (!ll || !log_ev || !log_dev || !log_wts || k < 1 || nlive <= k || ntot < nlive) return MCG_EINVAL;
  try {
    EvFold fold(nlive, k);
    const int64_t ndead = ntot - nlive;
    if (chunk > 0)
      for (int64_t a = std::min(chunk, ndead); a <= ndead; a = (a == ndead) ? ndead + 1 : std::min(a + chunk, ndead))
        fold.advance(ll, a, log_wts);
    fold.finish(ll, ntot, log_wts, log_ev, log_dev);
  } catch (const std::exception&) {
    return MCG_EFAIL;
  }
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
  // ascending ll; ties by concatenation index (= run, then position in the run)
  bool runs_sorted = true;
  for (int r = 0; r < nruns && runs_sorted; ++r)
    for (int64_t i = base[(size_t)r] + 1; i < base[(size_t)r + 1] && runs_sorted; ++i) runs_sorted = !(ll[i] < ll[i - 1]);
  if (runs_sorted && nruns > 1) {
    // nested outputs are already ascending: merge the runs pairwise (std::merge takes the first
    // range on ties, so the concatenation order of ties is kept) instead of sorting n indices
    std::vector<std::pair<double, int64_t>> a((size_t)n), b((size_t)n);
    for (int64_t p = 0; p < n; ++p) a[(size_t)p] = {ll[p], p};
    std::vector<int64_t> seg(base.begin(), base.end());
    auto less = [](const std::pair<double, int64_t>& x, const std::pair<double, int64_t>& y) { return x.first < y.first; };
    while (seg.size() > 2) {
      std::vector<int64_t> nseg{0};
      for (size_t r = 0; r + 1 < seg.size(); r += 2) {
        const int64_t lo = seg[r], mid = seg[r + 1], hi = r + 2 < seg.size() ? seg[r + 2] : seg[r + 1];
        std::merge(a.begin() + lo, a.begin() + mid, a.begin() + mid, a.begin() + hi, b.begin() + lo, less);
        nseg.push_back(hi);
      }
      a.swap(b);
      seg.swap(nseg);
    }
    for (int64_t p = 0; p < n; ++p) order[p] = a[(size_t)p].second;
  } else {
    for (int64_t p = 0; p < n; ++p) order[p] = p;
    std::stable_sort(order, order + n, [&](int64_t x, int64_t y) { return ll[x] < ll[y]; });
  }
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
