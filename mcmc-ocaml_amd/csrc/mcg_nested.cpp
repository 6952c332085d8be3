// mcg_nested.cpp -- Nested.nested_evidence driver (placeholder, filled in next).
#include "mcg_runtime.h"
using namespace mcg;
extern "C" {
int mcg_nested(mcg_ctx* ctx, const mcg_nested_opts* opts, mcg_nested_result* res,
               mcg_observer_fn observer, void* user) {
  (void)opts; (void)res; (void)observer; (void)user;
  return set_error(ctx, MCG_EINVAL, "nested sampling not built yet");
}
int mcg_nested_get(mcg_ctx* ctx, double* pts, double* ll, double* lp, double* log_wts) {
  (void)pts; (void)ll; (void)lp; (void)log_wts;
  return set_error(ctx, MCG_ESTATE, "no nested run");
}
}
