// mcg_device.h -- shared host/device declarations for the sampler kernels (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mcg {

// One kD-tree node, 16 B (one dwordx4 load per level).  Internal: dim >= 0, left child is the
// next node (pre-order), right child index in `right`.  Leaf: dim = -1 - leaf_index.
struct KdNode {
  double split;
  int32_t dim;
  int32_t right;
};

enum : int32_t { RUNF_RECORD_X = 1, RUNF_RECORD_LLP = 2, RUNF_RECORD_ACCEPT = 4, RUNF_ACCUMULATE = 8,
                 RUNF_RECORD_INITIAL = 16 };

// device view of one flattened kD tree (mcg_kdtree.cpp)
struct KdView {
  const KdNode* nodes;
  const double* logq;
  const double* box;
  const double* root;
  const int32_t* pt_leaf;
  int64_t M;
};

// Arguments of one MH launch (a contiguous slice of the steps of one mcg_run).
struct MhArgs {
  double* x;            // [D][N] chain state
  double* ll;           // [N]
  double* lp;           // [N]
  unsigned long long* nacc;  // [N] accepted-step counters (mcmc.ml:27-35)
  double* mean;         // [D][N] Welford accumulators over recorded samples
  double* m2;           // [D][N]
  double* hm_m;         // [8][N] log-space harmonic-mean partials of the record classes R & 7:
  double* hm_s;         // [8][N]   max of -ll and sum exp(-ll - max) (s == 0: empty class)
  double* rec_x;        // [n_rec][D][N]
  double* rec_ll;       // [n_rec][N]
  double* rec_lp;       // [n_rec][N]
  uint8_t* bits;        // [nsteps][bits_row_bytes] accept bitmap of the run
  const double* lik;    // likelihood constants (layout: mcg_runtime.cpp build_device_model)
  const double* pri;    // lo[D], hi[D], lp_in
  const double* prop;   // GAUSS: s[D]; WRAP: lo[D], hi[D], dx[D]
  const KdNode* kd_nodes;
  const double* kd_logq;   // [nleaves] log(n_leaf / (vol M))
  const double* kd_box;    // [nleaves][2][D]
  const double* kd_pts;    // [M][D]
  const double* kd_root;   // [2][D]
  const int32_t* kd_pt_leaf;  // [M] leaf of each training point
  int64_t kd_M;
  const double* de_pts;    // DE proposal samples [M][D] (differential_evolution_proposal)
  int64_t de_M;
  int64_t N;
  int64_t bits_row_bytes;
  uint64_t step_base;   // global (RNG) step index of this launch's first step
  int64_t t0;           // run-local index of this launch's first step
  int64_t nsteps;       // steps in this launch
  int64_t nskip;
  int64_t next_rec;     // run-local step count after which the next record is taken
  int64_t next_r;       // absolute record index of that record
  int64_t rec_end;      // absolute record index bound (exclusive)
  int64_t rec_base;     // absolute index of this run's record 0 (storage index = r - rec_base)
  const double* inv_n;  // inv_n[R - next_r0] = 1/(R+1) for the records of this launch
  int64_t next_r0;      // first record index covered by inv_n
  int64_t data_n;       // GAUSS_DATA / CAUCHY_DATA: number of data rows
  uint32_t k0, k1;      // Philox key = seed
  uint32_t chain_offset;
  int32_t prior_kind;
  int32_t flags;        // RUNF_*
  int32_t is_cauchy;
  int32_t uni;          // isotropic Gaussian proposal and one box for every dim (fused step only)
  int32_t ubox;         // one box [box_lo, box_hi] for every dim (any proposal; eval_prior)
  double uni_s, uni_lo, uni_hi;
  double box_lo, box_hi;
  // reversible jump (mcg_rj_kernel.h): model descriptors, tags, recorded tags, B-record counts
  const double* rj;
  uint8_t* tag;                 // [N]
  uint8_t* rec_tag;             // [n_rec][N]
  unsigned long long* rj_nb;    // [N] recorded samples in model B
  KdView rj_kd[2];
};

struct TileArgs {
  const double* mean; const double* m2; const double* hm_m; const double* hm_s;
  double* tiles;        // [ntiles][2D+3]
  int64_t N; int64_t nrec; int32_t D;
};

// kernel launchers (mcg_kernels_*.hip); return hipSuccess or an error
typedef hipError_t (*mh_launch_fn)(const MhArgs&, int64_t nthreads, hipStream_t);
mh_launch_fn find_mh_kernel(int D, int P, int lik, int prop);
typedef hipError_t (*eval_launch_fn)(const MhArgs&, hipStream_t);
eval_launch_fn find_eval_kernel(int D, int lik);
hipError_t launch_tile_stats(const TileArgs&, hipStream_t);
hipError_t launch_posterior_draw(const double* sums, int64_t npts, int64_t n, uint32_t k0, uint32_t k1,
                                 uint32_t call, int64_t* idx, hipStream_t);

}  // namespace mcg
