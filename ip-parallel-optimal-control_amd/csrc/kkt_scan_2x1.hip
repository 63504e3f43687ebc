// Instantiation unit of the KKT scan for (nx, nu) = (2, 1); see kkt_scan_impl.h.
#include "kkt_scan_impl.h"

namespace noc {
template <>
hipError_t kkt_dispatch_shape<2, 1>(const KKTArgs& a, int lanes, hipStream_t stream) {
  return dispatch_aff<2, 1>(a, lanes, stream);
}
}  // namespace noc
