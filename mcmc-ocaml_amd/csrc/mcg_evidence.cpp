// mcg_evidence.cpp -- kD-tree evidence integrals over MCMC output: Evidence.Make(MO)
// .evidence_direct and .evidence_lebesgue (evidence.ml:148-221) on the host.
//
// Both integrate over the cells of a Kd_tree built from the samples (kd_tree.ml:155-175) and
// stop descending at cells holding fewer than n samples (collect_subvolumes, evidence.ml:80-86).
// Only the cell object lists matter (the integrals use the objects' own bounding boxes), so the
// tree is never materialised: the recursion partitions index lists stably (List.partition keeps
// order, which fixes the order of every floating-point sum) and emits the collected cells in
// the reference's order, rev (cells of left) @ cells of right (List.rev_append, evidence.ml:85).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "mcg.h"

namespace {

struct Samples {
  int D;
  const double* x;   // [n][D]
  const double* ll;
  const double* lp;
  const double* c(int64_t i) const { return x + i * D; }
};

using Idx = std::vector<int64_t>;

// Pervasives.compare on float coordinates (lexicographic; NaN is not supported)
int cmp_coords(const Samples& s, int64_t a, int64_t b) {
  const double* p = s.c(a);
  const double* q = s.c(b);
  for (int d = 0; d < s.D; ++d) {
    if (p[d] < q[d]) return -1;
    if (p[d] > q[d]) return 1;
  }
  return 0;
}

// Kd.bounds_of_objects (kd_tree.ml:93-106)
void bounds(const Samples& s, const Idx& o, std::vector<double>& lo, std::vector<double>& hi) {
  lo.assign(s.c(o[0]), s.c(o[0]) + s.D);
  hi = lo;
  for (size_t k = 1; k < o.size(); ++k) {
    const double* p = s.c(o[k]);
    for (int d = 0; d < s.D; ++d) {
      if (p[d] < lo[(size_t)d]) lo[(size_t)d] = p[d];
      if (p[d] > hi[(size_t)d]) hi[(size_t)d] = p[d];
    }
  }
}

// Kd.bounds_volume (kd_tree.ml:177-182)
double volume(const std::vector<double>& lo, const std::vector<double>& hi) {
  double v = 1.0;
  for (size_t d = 0; d < lo.size(); ++d) v = v * (hi[d] - lo[d]);
  return v + 0.0;
}

// collect_subvolumes nmax (tree_of_objects objs ...) without building the tree
void collect(const Samples& s, const Idx& objs, int64_t nmax, std::vector<Idx>& out) {
  const int64_t n = (int64_t)objs.size();
  if (n == 0) return;                                   // Empty
  if (n < nmax) {                                       // not (length_at_least nmax objs)
    out.push_back(objs);
    return;
  }
  bool same = true;                                     // kd_tree.ml:158-159: a leaf cell
  for (int64_t k = 1; k < n && same; ++k) same = cmp_coords(s, objs[0], objs[(size_t)k]) == 0;
  if (n == 1 || same) return;                           // its Empty children collect nothing
  std::vector<double> lo, hi;
  bounds(s, objs, lo, hi);
  int dim = -1;                                         // longest_dim (kd_tree.ml:120-130)
  double dxm = -HUGE_VAL;
  for (int d = 0; d < s.D; ++d) {
    const double dx = hi[(size_t)d] - lo[(size_t)d];
    if (dx > dxm) { dim = d; dxm = dx; }
  }
  // find_ith: the (n/2)-th order statistic along dim (a unique value)
  std::vector<double> v((size_t)n);
  for (int64_t k = 0; k < n; ++k) v[(size_t)k] = s.c(objs[(size_t)k])[dim];
  std::nth_element(v.begin(), v.begin() + n / 2, v.end());
  const double pvt = v[(size_t)(n / 2)];
  Idx lte, gt;
  for (int64_t o : objs) (s.c(o)[dim] <= pvt ? lte : gt).push_back(o);
  if (gt.empty()) {                                     // adjust_for_empty_split (kd_tree.ml:144-153)
    double mx = s.c(lte[0])[dim];
    for (int64_t o : lte) mx = std::max(mx, s.c(o)[dim]);
    Idx a, b;
    for (int64_t o : lte) (s.c(o)[dim] < mx ? a : b).push_back(o);
    lte.swap(a);
    gt.swap(b);
  }
  std::vector<Idx> L, R;
  collect(s, lte, nmax, L);
  collect(s, gt, nmax, R);
  for (auto it = L.rbegin(); it != L.rend(); ++it) out.push_back(std::move(*it));
  for (auto& c : R) out.push_back(std::move(c));
}

}  // namespace

extern "C" {

int mcg_evidence_direct(int32_t ndim, int64_t n, const double* pts, const double* ll, const double* lp,
                        int64_t nbox, double* out) {
  if (ndim < 1 || n < 1 || !pts || !ll || !lp || !out) return MCG_EINVAL;
  const Samples s{ndim, pts, ll, lp};
  // array_to_list_remove_dups (evidence.ml:140-143): stable sort by coordinates, keep the last
  // of each run of equal points, reversed
  Idx idx((size_t)n);
  for (int64_t i = 0; i < n; ++i) idx[(size_t)i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return cmp_coords(s, a, b) < 0; });
  Idx u;
  for (size_t k = 0; k < idx.size(); ++k)
    if (k + 1 == idx.size() || cmp_coords(s, idx[k], idx[k + 1]) != 0) u.push_back(idx[k]);
  std::reverse(u.begin(), u.end());
  std::vector<Idx> cells;
  collect(s, u, nbox, cells);
  // evidence_direct_tree (evidence.ml:145-156): sum of vol * mean posterior over the cells
  double integral = 0.0;
  std::vector<double> lo, hi;
  for (const Idx& c : cells) {
    bounds(s, c, lo, hi);
    const double vol = volume(lo, hi);
    double sum = 0.0;
    for (int64_t o : c) sum = sum + std::exp(ll[o] + lp[o]);
    integral = integral + vol * (sum / (double)c.size());
  }
  *out = integral;
  return MCG_OK;
}

int mcg_evidence_lebesgue(int32_t ndim, int64_t n, const double* pts, const double* ll, const double* lp,
                          int64_t nbox, double eps, double* out) {
  if (ndim < 1 || n < 1 || !pts || !ll || !lp || !out) return MCG_EINVAL;
  const Samples s{ndim, pts, ll, lp};
  // collect_samples_up_to_eps (evidence.ml:158-172): ascending 1/L (stable), the prefix whose
  // consecutive gaps in 1/L are <= eps, plus the sample before the first larger gap
  Idx idx((size_t)n);
  for (int64_t i = 0; i < n; ++i) idx[(size_t)i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return -ll[a] < -ll[b]; });
  Idx col;
  for (size_t k = 0; k < idx.size(); ++k) {
    col.push_back(idx[k]);
    if (k + 1 < idx.size() && std::exp(-ll[idx[k + 1]]) - std::exp(-ll[idx[k]]) > eps) break;
  }
  // mean_inv_like (evidence.ml:174-181)
  double til = 0.0;
  for (int64_t o : col) til = til + std::exp(-ll[o]);
  const double mean_il = til / (double)col.size();
  // remove_dups_rev (evidence.ml:183-192): drop x when ll x = ll (next), reversed
  Idx u;
  for (size_t k = 0; k < col.size(); ++k)
    if (k + 1 == col.size() || ll[col[k]] != ll[col[k + 1]]) u.push_back(col[k]);
  std::reverse(u.begin(), u.end());
  std::vector<Idx> cells;
  collect(s, u, nbox, cells);
  // prior mass: sum of vol * exp (median log_prior) over the cells (evidence.ml:200-211)
  double pm = 0.0;
  std::vector<double> lo, hi;
  for (const Idx& c : cells) {
    bounds(s, c, lo, hi);
    const double vol = volume(lo, hi);
    Idx o = c;
    std::stable_sort(o.begin(), o.end(), [&](int64_t a, int64_t b) { return lp[a] < lp[b]; });
    const size_t m = o.size();
    const double med = (m % 2 == 0) ? 0.5 * (lp[o[m / 2 - 1]] + lp[o[m / 2]]) : lp[o[m / 2]];
    pm = pm + std::exp(med) * vol;
  }
  *out = pm / mean_il;
  return MCG_OK;
}

}  // extern "C"
