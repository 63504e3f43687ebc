// Instantiation unit of the KKT scan for a registered custom family's (nx, nu) -- compiled only by
// a custom-family build (noc.families.register_family), which passes NOC_CUSTOM_NX / NOC_CUSTOM_NU.
#include "../kkt_scan_impl.h"

namespace noc {
template <>
hipError_t kkt_dispatch_shape<NOC_CUSTOM_NX, NOC_CUSTOM_NU>(const KKTArgs& a, int lanes,
                                                            hipStream_t stream) {
  return dispatch_aff<NOC_CUSTOM_NX, NOC_CUSTOM_NU>(a, lanes, stream);
}
}  // namespace noc
