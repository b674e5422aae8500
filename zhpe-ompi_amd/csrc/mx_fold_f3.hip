// mx_fold_f3.hip -- instantiates the fold kernels (mx_fold.hpp) for
// element-type family 3 only; the families are split over translation units
// so the kernel library builds in parallel.
#include "mx_fold.hpp"

namespace mx {
FoldFns fold_fns_fam3(int op, int type) {
  FamVisitor<3> v;
  return dispatch(op, type, v);
}
}  // namespace mx
