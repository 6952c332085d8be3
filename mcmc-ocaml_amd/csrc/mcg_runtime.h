// mcg_runtime.h -- internal host-side state of a sampling context.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <sys/mman.h>

#include "mcg.h"
#include "mcg_device.h"

namespace mcg {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf();
  hipError_t ensure(size_t n);
  void release();
};

struct KdState {
  bool built = false;
  int64_t M = 0;
  int64_t nnodes = 0, nleaves = 0;
  std::vector<KdNode> nodes;
  std::vector<double> logq, box, pts, root;
  std::vector<int32_t> count, pt_leaf;
  DevBuf d_nodes, d_logq, d_box, d_pts, d_root, d_pt_leaf;
};

// A growable host array of doubles in malloc'd memory, so a finished run's arrays can be handed to
// the caller without a copy (mcg_nested_take; the caller frees them with mcg_free).  No element is
// initialised by resize (every element is written before it is read); growth is realloc (an
// mremap for large blocks: no copy).
class HostArr {
 public:
  HostArr() = default;
  HostArr(const HostArr&) = delete;
  HostArr& operator=(const HostArr&) = delete;
  ~HostArr() { std::free(p_); }
  size_t size() const { return n_; }
  size_t capacity() const { return cap_; }
  double* data() { return p_; }
  const double* data() const { return p_; }
  double& operator[](size_t i) { return p_[i]; }
  double operator[](size_t i) const { return p_[i]; }
  void clear() { n_ = 0; }
  bool reserve(size_t c) {
    if (c <= cap_) return true;
    void* q = std::realloc(p_, c * sizeof(double));
    if (!q) return false;
    p_ = (double*)q;
    cap_ = c;
    return true;
  }
  bool resize(size_t n) {
    if (n > cap_ && !reserve(std::max(n, 2 * cap_))) return false;
    n_ = n;
    return true;
  }
  bool append(const double* a, const double* b) {
    const size_t m = (size_t)(b - a);
    if (!resize(n_ + m)) return false;
    std::memcpy(p_ + n_ - m, a, m * sizeof(double));
    return true;
  }
  // an empty array's first block: 2 MiB aligned (transparent huge pages), not yet touched
  bool reserve_fresh(size_t c) {
    if (p_ || c == 0) return reserve(c);
    const size_t bytes = ((c * sizeof(double)) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    void* q = std::aligned_alloc((size_t)2 << 20, bytes);
    if (!q) return false;
    (void)madvise(q, bytes, MADV_HUGEPAGE);
    p_ = (double*)q;
    cap_ = bytes / sizeof(double);
    return true;
  }
  double* release() {                       // ownership to the caller (free)
    double* q = p_;
    p_ = nullptr;
    n_ = cap_ = 0;
    return q;
  }

 private:
  double* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
};

struct NestedState {
  // last run: ll, lp, wts of every point (dead in retirement order, then live ascending); the
  // rows of every point stay in the device dead buffer (the live rows gathered behind the dead)
  HostArr ll, lp, wts;
  bool taken = false;                     // ll / lp / wts handed to the caller (mcg_nested_take)
  // after a take: the next run's fresh blocks are prefaulted (MADV_POPULATE_WRITE, which leaves
  // their contents alone, so the run may write them meanwhile); joined before any reallocation
  std::thread populate;
  void join_populate() {
    if (populate.joinable()) populate.join();
  }
  ~NestedState() { join_populate(); }
  double wts_shift = 0.0;                 // wts hold log weights + log Z; mcg_nested_get subtracts it
  int64_t n_total = 0, n_dead = 0, n_gen = 0, nlive = 0, ndim = 0;
  int64_t ndim_k = 0;                     // the device rows' width (ndim zero-padded)
  double log_ev = 0.0, log_dev = 0.0;
  bool converged = false;       // the stop test fired (false: max_dead reached first)
};

}  // namespace mcg

struct mcg_nested_bufs_holder;
void mcg_free_nested_bufs(mcg_nested_bufs_holder* h);

struct mcg_ctx {
  mcg_opts opts{};
  std::string err;
  std::string arch;
  int num_cus = 256;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // model: D = the caller's ndim; Dk = the compiled width the kernels run at (D <= Dk, the dims
  // D..Dk-1 zero-padded on the device and stripped at every copy out; pad_width)
  int D = 0;
  int Dk = 0;
  int32_t lik_kind = -1, prior_kind = MCG_PRIOR_FLAT, prop_kind = MCG_PROP_GAUSS;
  uint64_t state_token = 0;              // bumped by every state-changing entry point (mcg_state_token)
  int32_t is_cauchy = 0;
  int64_t data_n = 0;
  std::vector<double> lik_host, pri_host, prop_host;
  // the caller's (unpadded) prior and proposal parameters: re-laid out at a new kernel width when
  // a likelihood of another kind pads the same ndim differently (prop_raw_kind -1: a proposal
  // that cannot be re-laid out from parameters alone -- kD tree, DE samples)
  int32_t prior_raw_kind = MCG_PRIOR_FLAT, prop_raw_kind = -1;
  std::vector<double> prior_raw, prop_raw;
  mcg::DevBuf d_lik, d_pri, d_prop;
  mcg::KdState kd;
  mcg::DevBuf d_de_pts;          // differential_evolution_proposal samples [M][D]
  int64_t de_M = 0;
  int de_D = 0;
  // chains
  int64_t N = 0;
  mcg::DevBuf d_x, d_ll, d_lp, d_nacc;
  uint64_t steps_done = 0;      // global RNG step counter (all runs)
  uint32_t post_calls = 0;      // mcg_posterior_samples calls since create / reseed
  int64_t nsteps_total = 0;     // steps of the current chains since init / the last counter reset
  uint64_t acc_base = 0, rej_base = 0;  // tallies of earlier chain sets (folded at mcg_init)
  int64_t last_nsteps = 0;
  int lanes = 1;
  // records and statistics
  mcg::DevBuf d_rec_x, d_rec_ll, d_rec_lp, d_bits, d_mean, d_m2, d_hm_m, d_hm_s, d_tiles;
  int64_t nrec_total = 0, rec_stored = 0;
  mcg::DevBuf d_invtab;                  // Welford weights 1/(R+1), R = absolute record index
  int64_t inv_cap = 0;
  bool rec_x_valid = false, rec_llp_valid = false, last_record_accept = false;
  // reversible jump (mcg_rj.cpp)
  bool rj_active = false;
  std::vector<double> rj_host;
  mcg::DevBuf d_rj, d_tag, d_rec_tag, d_rj_nb;
  mcg::KdState rj_kd[2];
  std::vector<double> rj_root[2];
  mcg::DevBuf d_rj_root[2];
  // nested sampling
  mcg::NestedState nested;
  mcg_nested_bufs_holder* nested_bufs = nullptr;
  // timing: per-launch HIP event pairs on the launch stream, harvested lazily (no host sync
  // inside mcg_run)
  bool timing = false;
  mcg_kernel_timing t_mh{}, t_walk{};
  int64_t t_mh_steps = 0;
  std::vector<hipEvent_t> ev_free;
  struct Pending { hipEvent_t a, b; int kind; };
  std::vector<Pending> ev_pending;
};

namespace mcg {
int set_error(mcg_ctx* ctx, int code, const char* fmt, ...);
int hip_check(mcg_ctx* ctx, hipError_t e, const char* what);
int quiesce(mcg_ctx* ctx);
int fold_counters(mcg_ctx* ctx);
MhArgs base_args(mcg_ctx* ctx);
int choose_lanes(mcg_ctx* ctx);
double host_pexp(double x);
void timing_begin(mcg_ctx* ctx, hipEvent_t* a, hipEvent_t* b);
void timing_end(mcg_ctx* ctx, hipEvent_t a, hipEvent_t b, int kind);
void timing_harvest(mcg_ctx* ctx);
int kd_build(mcg_ctx* ctx, const double* pts, int64_t M, int D, const double* low, const double* high,
             KdState* dst = nullptr, int Dpad = 0);
int pack_likelihood(mcg_ctx* ctx, int32_t kind, int D, const double* params, size_t n,
                    std::vector<double>& dev, int32_t* is_cauchy, int64_t* data_n);
int pack_prior(mcg_ctx* ctx, int32_t kind, int D, const double* params, size_t n, std::vector<double>& dev);
// Zero padding of a model to a compiled width DM >= D (mcg.h "Any ndim"): a padded dim holds 0 for
// the whole run and adds +0 to every canonical sum, so the real dims compute exactly as at D.
// The smallest compiled width >= D for a likelihood kind (D itself when it is compiled or when no
// compiled width is larger)
int pad_width(int32_t lik_kind, int D);
// a likelihood block packed at D laid out at DM (zeros)
std::vector<double> pad_lik(int32_t kind, int D, int DM, const std::vector<double>& v);
// a prior block [check_lo, check_hi, lp_in, lo, hi] packed at D laid out at DM: padded dims
// unbounded in the check and drawn in [pad_draw, pad_draw] (0: nested sampling's prior draws
// leave them at 0)
std::vector<double> pad_prior(int D, int DM, const std::vector<double>& v, double pad_draw_lo, double pad_draw_hi);
// a DIAG_GAUSS prior descriptor at width DM: zero constants (and mu = sigma = 0) in the pad dims
std::vector<double> pad_gauss_prior(int D, int DM, const std::vector<double>& v);
// rows [n][D] -> [n][DM] with zero pad columns
std::vector<double> pad_rows(const double* rows, int64_t n, int D, int DM);
typedef hipError_t (*rj_init_fn)(const MhArgs&, int draw_tags, const double* xa, const double* xb, hipStream_t);
mh_launch_fn find_rj_kernel(int DM);
rj_init_fn find_rj_init(int DM);
void rj_args(mcg_ctx* ctx, MhArgs& a);
}  // namespace mcg
