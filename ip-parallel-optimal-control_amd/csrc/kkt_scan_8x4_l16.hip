// Instantiation unit of the KKT scan for (nx, nu) = (8, 4), lanes 16 (see kkt_scan_8x4.hip).
#include "kkt_scan_impl.h"

namespace noc {
template hipError_t launch_kkt<8, 4, 16, true>(const KKTArgs&, hipStream_t);
template hipError_t launch_kkt<8, 4, 16, false>(const KKTArgs&, hipStream_t);
}  // namespace noc
