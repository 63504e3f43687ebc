// Instantiation unit of the horizon-sequential group KKT solve (lanes = 1); see kkt_group_impl.h.
#include "kkt_group8_impl.h"

namespace noc {
hipError_t kkt_group_dispatch(int nx, int nu, const KKTArgs& a, hipStream_t stream) {
  if (nx == 2 && nu == 1) return launch_kkt_group<2, 1>(a, stream);
  if (nx == 4 && nu == 1) return launch_kkt_group<4, 1>(a, stream);
  if (nx == 8 && nu == 4) return launch_kkt_group8(a, stream);
  return hipErrorInvalidValue;
}
}  // namespace noc
