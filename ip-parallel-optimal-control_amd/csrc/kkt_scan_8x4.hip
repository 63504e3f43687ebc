// Instantiation unit of the KKT scan for (nx, nu) = (8, 4); see kkt_scan_impl.h.
#include "kkt_scan_impl.h"

namespace noc {
template <>
hipError_t kkt_dispatch_shape<8, 4>(const KKTArgs& a, int lanes, hipStream_t stream) {
  return dispatch_aff<8, 4>(a, lanes, stream);
}
}  // namespace noc
