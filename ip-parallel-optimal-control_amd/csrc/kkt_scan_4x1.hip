// Instantiation unit of the KKT scan for (nx, nu) = (4, 1); see kkt_scan_impl.h.
#include "kkt_scan_impl.h"

namespace noc {
hipError_t kkt_dispatch_4x1(const KKTArgs& a, int lanes, hipStream_t stream) {
  return dispatch_aff<4, 1>(a, lanes, stream);
}
}  // namespace noc
