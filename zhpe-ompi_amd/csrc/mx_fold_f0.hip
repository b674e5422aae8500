// mx_fold_f0.hip -- instantiates the fold kernels (mx_fold.hpp) for
// element-type family 0 only; the families are split over translation units
// so the kernel library builds in parallel.
#include "mx_fold.hpp"

namespace mx {
FoldFns fold_fns_fam0(int op, int type) {
  FamVisitor<0> v;
  return dispatch(op, type, v);
}
}  // namespace mx
