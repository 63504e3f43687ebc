// Instantiation unit of the KKT scan for (nx, nu) = (8, 4), lanes 64; see kkt_scan_impl.h.  The
// other lane counts are compiled in parallel units (kkt_scan_8x4_l*.hip): the nx = 8 element's
// unrolled combine makes one unit with every instance the slowest step of the build.
#include "kkt_scan_impl.h"

namespace noc {
extern template hipError_t launch_kkt<8, 4, 32, true>(const KKTArgs&, hipStream_t);
extern template hipError_t launch_kkt<8, 4, 32, false>(const KKTArgs&, hipStream_t);
extern template hipError_t launch_kkt<8, 4, 16, true>(const KKTArgs&, hipStream_t);
extern template hipError_t launch_kkt<8, 4, 16, false>(const KKTArgs&, hipStream_t);
extern template hipError_t launch_kkt<8, 4, 8, true>(const KKTArgs&, hipStream_t);
extern template hipError_t launch_kkt<8, 4, 8, false>(const KKTArgs&, hipStream_t);

template <>
hipError_t kkt_dispatch_shape<8, 4>(const KKTArgs& a, int lanes, hipStream_t stream) {
  return dispatch_aff<8, 4>(a, lanes, stream);
}
}  // namespace noc
