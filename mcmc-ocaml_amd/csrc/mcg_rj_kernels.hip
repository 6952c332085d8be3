// mcg_rj_kernels.hip -- instantiations of the reversible-jump kernels (mcg_rj_kernel.h) for
// max(D_A, D_B) in 1..8, 16, 32.
#include "mcg_rj_kernel.h"
#include "mcg_runtime.h"

namespace mcg {

#define MCG_RJ_DIMS(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(16) X(32)

mh_launch_fn find_rj_kernel(int DM) {
#define MCG_RJ_CASE(n) \
  if (DM == n) return &launch_rj<n>;
  MCG_RJ_DIMS(MCG_RJ_CASE)
#undef MCG_RJ_CASE
  return nullptr;
}

rj_init_fn find_rj_init(int DM) {
#define MCG_RJ_CASE(n) \
  if (DM == n) return &launch_rj_init<n>;
  MCG_RJ_DIMS(MCG_RJ_CASE)
#undef MCG_RJ_CASE
  return nullptr;
}

}  // namespace mcg
