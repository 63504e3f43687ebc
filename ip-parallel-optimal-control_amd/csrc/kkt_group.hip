// Instantiation unit of the horizon-sequential group KKT solve (lanes = 1); see kkt_group_impl.h.
#include "kkt_group8_impl.h"

namespace noc {
// one nx-lane group per trajectory: shapes of kkt_shapes.def with nx | 64 and nu <= nx; (8, 4)
// runs the LDS-DMA-staged nx = 8 kernel (kkt_group8_impl.h).  A template, so the shapes without a
// group kernel are never instantiated.
template <int X, int U>
static hipError_t group_shape(const KKTArgs& a, hipStream_t stream) {
  if constexpr (X == 8 && U == 4) return launch_kkt_group8(a, stream);
  else if constexpr (64 % X == 0 && U <= X) return launch_kkt_group<X, U>(a, stream);
  else return hipErrorInvalidValue;
}

hipError_t kkt_group_dispatch(int nx, int nu, const KKTArgs& a, hipStream_t stream) {
#define NOC_KKT_SHAPE(X, U) if (nx == X && nu == U) return group_shape<X, U>(a, stream);
#include NOC_KKT_SHAPES_DEF
#undef NOC_KKT_SHAPE
  return hipErrorInvalidValue;
}
}  // namespace noc
