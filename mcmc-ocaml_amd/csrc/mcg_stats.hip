// mcg_stats.hip -- tile reduction of the per-chain accumulators.
//
// One 256-thread workgroup per 256-chain tile.  Per dim, the entries (n, mean_d, m2_d) are
// combined by the Chan et al. pairwise update in a fixed LDS tree (stride 128, 64, ..., 1);
// the harmonic-mean partials (max, sum) by a log-space combine in the same tree.  The tree is
// fixed, so tile partials are bit-identical to the oracle's (oracle.c or_tile_stats) and do not
// depend on how many GPUs share the chains.  Multi_mean / multi_std (stats.ml:58-87) and
// evidence_harmonic_mean (evidence.ml:101-107) are finished on the host from the tiles.
#include "mcg_device.h"
#include "mcg_math.h"

namespace mcg {

__global__ void __launch_bounds__(256) tile_stats_kernel(const TileArgs a) {
  __shared__ double sn[256], sm[256], s2[256];
  const int t = threadIdx.x;
  const int64_t c = (int64_t)blockIdx.x * 256 + t;
  const bool valid = c < a.N && a.nrec > 0;
  const int D = a.D;
  double* out = a.tiles + (int64_t)blockIdx.x * (2 * D + 3);
  for (int d = 0; d < D; ++d) {
    sn[t] = valid ? (double)a.nrec : 0.0;
    sm[t] = valid ? a.mean[(int64_t)d * a.N + c] : 0.0;
    s2[t] = valid ? a.m2[(int64_t)d * a.N + c] : 0.0;
    __syncthreads();
    for (int s = 128; s >= 1; s >>= 1) {
      if (t < s) {
        double na = sn[t], nb = sn[t + s];
        if (nb != 0.0) {
          if (na == 0.0) {
            sn[t] = nb; sm[t] = sm[t + s]; s2[t] = s2[t + s];
          } else {
            double n = na + nb;
            double fb = nb / n;
            double fab = (na * nb) / n;
            double delta = sm[t + s] - sm[t];
            sm[t] = sm[t] + delta * fb;
            s2[t] = (s2[t] + s2[t + s]) + (delta * delta) * fab;
            sn[t] = n;
          }
        }
      }
      __syncthreads();
    }
    if (t == 0) {
      out[0] = sn[0];
      out[1 + d] = sm[0];
      out[1 + D + d] = s2[0];
    }
    __syncthreads();
  }
  // harmonic-mean partials: the chain's 8 record classes in the canonical tree
  // ((0,4),(2,6)),((1,5),(3,7)) (oracle.c hm_classes), then the tile tree
  double hm = -__builtin_inf(), hs = 0.0;
  if (valid) {
    double cm[8], cs[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { cm[k] = a.hm_m[(int64_t)k * a.N + c]; cs[k] = a.hm_s[(int64_t)k * a.N + c]; }
#pragma unroll
    for (int k = 0; k < 4; ++k) hm_comb(cm[k], cs[k], cm[k + 4], cs[k + 4]);
    hm_comb(cm[0], cs[0], cm[2], cs[2]);
    hm_comb(cm[1], cs[1], cm[3], cs[3]);
    hm_comb(cm[0], cs[0], cm[1], cs[1]);
    hm = cm[0]; hs = cs[0];
  }
  sn[t] = valid ? 1.0 : 0.0;
  sm[t] = hm;
  s2[t] = hs;
  __syncthreads();
  for (int s = 128; s >= 1; s >>= 1) {
    if (t < s) {
      double na = sn[t], nb = sn[t + s];
      if (nb != 0.0) {
        if (na == 0.0) {
          sn[t] = nb; sm[t] = sm[t + s]; s2[t] = s2[t + s];
        } else {
          double ma = sm[t], mb = sm[t + s];
          double mm = (ma > mb) ? ma : mb;
          s2[t] = s2[t] * pexp(ma - mm) + s2[t + s] * pexp(mb - mm);
          sm[t] = mm;
          sn[t] = na + nb;
        }
      }
    }
    __syncthreads();
  }
  if (t == 0) {
    if (D == 0) out[0] = valid ? (double)a.nrec : 0.0;
    out[2 * D + 1] = sm[0];
    out[2 * D + 2] = s2[0];
  }
}

hipError_t launch_tile_stats(const TileArgs& a, hipStream_t s) {
  const int64_t ntiles = (a.N + 255) / 256;
  hipLaunchKernelGGL(tile_stats_kernel, dim3((unsigned)ntiles), dim3(256), 0, s, a);
  return hipGetLastError();
}

// Nested.posterior_samples (nested.ml:167-178): one thread per draw, u = Random.float 1.0 from
// Philox (i lo, i hi, call, tag 5), then weight_binary_search_index (nested.ml:152-165) over the
// running sums (L2-resident; log2(npts) dependent loads per draw).
__global__ void __launch_bounds__(256) posterior_draw_kernel(const double* __restrict__ sums, int64_t npts,
                                                             int64_t n, uint32_t k0, uint32_t k1,
                                                             uint32_t call, int64_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const u32x4 w = philox((uint32_t)i, (uint32_t)((uint64_t)i >> 32), call, TAG_POSTERIOR << 16, k0, k1);
  const double x = u53(w.x, w.y);
  int64_t r;
  if (x <= sums[0]) {
    r = 0;
  } else {
    int64_t lo = 0, hi = npts - 1;
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) / 2;
      if (x <= sums[mid]) hi = mid;
      else lo = mid;
    }
    r = hi;
  }
  idx[i] = r;
}

hipError_t launch_posterior_draw(const double* sums, int64_t npts, int64_t n, uint32_t k0, uint32_t k1,
                                 uint32_t call, int64_t* idx, hipStream_t s) {
  if (n < 1) return hipSuccess;
  hipLaunchKernelGGL(posterior_draw_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, sums, npts,
                     n, k0, k1, call, idx);
  return hipGetLastError();
}

}  // namespace mcg
