// mcg_kdtree.cpp -- host build of the Farr-Mandel kD tree and its flattened HBM image.
//
// Kd_tree.tree_of_objects (kd_tree.ml:155-175): a cell holding more than one distinct point is
// split on the longest dimension of its points' bounding box (longest_dim, kd_tree.ml:120-130)
// at the n/2-th order statistic; lte = points <= pivot, gt = the rest (kd_tree.ml:162-168), with
// adjust_for_empty_split (kd_tree.ml:144-153) when gt is empty; the split plane is the midpoint
// of max(lte) and min(gt) (split_bounds, kd_tree.ml:112-118).  The reference finds the order
// statistic with a randomized quickselect (find_ith, kd_tree.ml:69-86); the value it returns is
// unique, so nth_element gives the same tree.  Each leaf stores log(n_leaf / (vol * M)), the
// log of Interpolate_pdf.jump_prob (interpolate_pdf.ml:135-142).
#include <algorithm>
#include <cmath>
#include <numeric>

#include "mcg_runtime.h"

namespace mcg {

namespace {

struct Builder {
  const double* pts;
  int D;
  int64_t M;
  std::vector<KdNode> nodes;
  std::vector<double> box, logq;
  std::vector<int32_t> count;

  double at(int64_t i, int d) const { return pts[i * D + d]; }

  int32_t leaf(int64_t n, const std::vector<double>& lo, const std::vector<double>& hi) {
    const int32_t L = (int32_t)count.size();
    count.push_back((int32_t)n);
    box.insert(box.end(), lo.begin(), lo.end());
    box.insert(box.end(), hi.begin(), hi.end());
    double v = 1.0;                                   // bounds_volume (kd_tree.ml:177-182)
    for (int d = 0; d < D; ++d) v = v * (hi[d] - lo[d]);
    v = v + 0.0;
    logq.push_back(std::log((double)n / (v * (double)M)));
    return L;
  }

  int32_t build(int64_t* idx, int64_t n, const std::vector<double>& lo, const std::vector<double>& hi) {
    const int32_t node = (int32_t)nodes.size();
    nodes.push_back(KdNode{0.0, -1, -1});
    bool all_eq = true;
    for (int64_t i = 1; i < n && all_eq; ++i)
      for (int d = 0; d < D; ++d)
        if (at(idx[i], d) != at(idx[0], d)) { all_eq = false; break; }
    if (n == 1 || all_eq) {
      nodes[node].dim = -1 - leaf(n, lo, hi);
      return node;
    }
    int dim = -1;
    double dmax = -HUGE_VAL;
    for (int d = 0; d < D; ++d) {
      double l = at(idx[0], d), h = l;
      for (int64_t i = 1; i < n; ++i) {
        const double c = at(idx[i], d);
        l = std::min(l, c);
        h = std::max(h, c);
      }
      if (h - l > dmax) { dmax = h - l; dim = d; }
    }
    auto key = [&](int64_t i) { return at(i, dim); };
    std::nth_element(idx, idx + n / 2, idx + n, [&](int64_t a, int64_t b) { return key(a) < key(b); });
    const double pv = key(idx[n / 2]);
    int64_t* mid = std::partition(idx, idx + n, [&](int64_t i) { return key(i) <= pv; });
    if (mid == idx + n) {
      double mx = -HUGE_VAL;
      for (int64_t i = 0; i < n; ++i) mx = std::max(mx, key(idx[i]));
      mid = std::partition(idx, idx + n, [&](int64_t i) { return key(i) < mx; });
    }
    const int64_t nlte = mid - idx;
    double lt = -HUGE_VAL, gt = HUGE_VAL;
    for (int64_t i = 0; i < nlte; ++i) lt = std::max(lt, key(idx[i]));
    for (int64_t i = nlte; i < n; ++i) gt = std::min(gt, key(idx[i]));
    const double x = 0.5 * (lt + gt);
    std::vector<double> nhi(hi), nlo(lo);
    nhi[dim] = x;
    nlo[dim] = x;
    nodes[node].dim = dim;
    nodes[node].split = x;
    build(idx, nlte, lo, nhi);
    const int32_t r = build(idx + nlte, n - nlte, nlo, hi);
    nodes[node].right = r;
    return node;
  }
};

}  // namespace

int kd_build(mcg_ctx* ctx, const double* pts, int64_t M, int D, const double* low,
             const double* high, KdState* dst, int Dpad) {
  Builder b{pts, D, M, {}, {}, {}, {}};
  std::vector<int64_t> idx((size_t)M);
  std::iota(idx.begin(), idx.end(), 0);
  std::vector<double> lo(low, low + D), hi(high, high + D);
  b.build(idx.data(), M, lo, hi);
  KdState& k = dst ? *dst : ctx->kd;
  k.M = M;
  k.nnodes = (int64_t)b.nodes.size();
  k.nleaves = (int64_t)b.count.size();
  k.nodes = std::move(b.nodes);
  k.logq = std::move(b.logq);
  k.box = std::move(b.box);
  k.count = std::move(b.count);
  k.pts.assign(pts, pts + M * D);
  k.root.assign(low, low + D);
  k.root.insert(k.root.end(), high, high + D);
  // leaf of every training point (Interpolate_pdf.draw's find_cell of the picked point,
  // interpolate_pdf.ml:114-119) -- the same descent as kd_find_leaf on the device
  k.pt_leaf.assign((size_t)M, 0);
  for (int64_t i = 0; i < M; ++i) {
    bool inside = true;
    for (int d = 0; d < D; ++d) inside = inside && pts[i * D + d] >= low[d] && pts[i * D + d] <= high[d];
    int32_t node = 0;
    while (k.nodes[(size_t)node].dim >= 0) {
      const KdNode& nd = k.nodes[(size_t)node];
      node = (inside && pts[i * D + nd.dim] <= nd.split) ? node + 1 : nd.right;
    }
    k.pt_leaf[(size_t)i] = -1 - k.nodes[(size_t)node].dim;
  }
  int rc;
  auto up = [&](DevBuf& d, const void* h, size_t bytes) {
    int r = hip_check(ctx, d.ensure(bytes), "alloc kd");
    if (r) return r;
    return hip_check(ctx, hipMemcpy(d.p, h, bytes, hipMemcpyHostToDevice), "copy kd");
  };
  if ((rc = up(k.d_nodes, k.nodes.data(), k.nodes.size() * sizeof(KdNode)))) return rc;
  if ((rc = up(k.d_logq, k.logq.data(), k.logq.size() * 8))) return rc;
  if (Dpad > D) {
    // the MH kernel of width Dpad (zero-padded model): leaf boxes and the root
    // box as [lo, hi] = [0, 0] in the pad dims, so a draw puts 0 there (the pad invariant) and
    // the descent's root test holds for it; log q stays the D-dim density of the caller's tree.
    // (A pad dim's draw is never strictly inside its box, so these kernels take the descent for
    // every proposal: the same leaf, a slower step.)
    std::vector<double> box((size_t)k.nleaves * 2 * Dpad, 0.0), root(2 * (size_t)Dpad, 0.0);
    for (int64_t l = 0; l < k.nleaves; ++l)
      for (int d = 0; d < D; ++d) {
        box[(size_t)l * 2 * Dpad + d] = k.box[(size_t)l * 2 * D + d];
        box[(size_t)l * 2 * Dpad + Dpad + d] = k.box[(size_t)l * 2 * D + D + d];
      }
    for (int d = 0; d < D; ++d) {
      root[d] = k.root[d];
      root[Dpad + d] = k.root[D + d];
    }
    if ((rc = up(k.d_box, box.data(), box.size() * 8))) return rc;
    if ((rc = up(k.d_root, root.data(), root.size() * 8))) return rc;
  } else {
    if ((rc = up(k.d_box, k.box.data(), k.box.size() * 8))) return rc;
    if ((rc = up(k.d_root, k.root.data(), k.root.size() * 8))) return rc;
  }
  if ((rc = up(k.d_pts, k.pts.data(), k.pts.size() * 8))) return rc;
  if ((rc = up(k.d_pt_leaf, k.pt_leaf.data(), k.pt_leaf.size() * 4))) return rc;
  k.built = true;
  return MCG_OK;
}

}  // namespace mcg

extern "C" {
// flattened tree of the last mcg_set_kd_proposal (for tests / tools): node_dim (-1 leaf),
// node_split, node_right, node_leaf, leaf_count, leaf_box [nl][2][D], leaf_logq
int mcg_kd_info(mcg_ctx* ctx, int64_t* nnodes, int64_t* nleaves) {
  if (!ctx) return MCG_EINVAL;
  if (nnodes) *nnodes = ctx->kd.nnodes;
  if (nleaves) *nleaves = ctx->kd.nleaves;
  return ctx->kd.built ? MCG_OK : MCG_ESTATE;
}

int mcg_kd_export(mcg_ctx* ctx, int32_t* node_dim, double* node_split, int32_t* node_right,
                  int32_t* node_leaf, int32_t* leaf_count, double* leaf_box, double* leaf_logq) {
  if (!ctx || !ctx->kd.built) return MCG_ESTATE;
  const auto& k = ctx->kd;
  for (int64_t i = 0; i < k.nnodes; ++i) {
    const mcg::KdNode& nd = k.nodes[(size_t)i];
    if (node_dim) node_dim[i] = nd.dim >= 0 ? nd.dim : -1;
    if (node_split) node_split[i] = nd.dim >= 0 ? nd.split : 0.0;
    if (node_right) node_right[i] = nd.dim >= 0 ? nd.right : -1;
    if (node_leaf) node_leaf[i] = nd.dim >= 0 ? -1 : -1 - nd.dim;
  }
  if (leaf_count) std::copy(k.count.begin(), k.count.end(), leaf_count);
  if (leaf_box) std::copy(k.box.begin(), k.box.end(), leaf_box);
  if (leaf_logq) std::copy(k.logq.begin(), k.logq.end(), leaf_logq);
  return MCG_OK;
}
}
