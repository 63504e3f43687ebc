// Instantiation unit of the KKT scan for (nx, nu) = (4, 1), lanes 32 (see kkt_scan_4x1.hip).
#include "kkt_scan_impl.h"

namespace noc {
template hipError_t launch_kkt<4, 1, 32, true>(const KKTArgs&, hipStream_t);
template hipError_t launch_kkt<4, 1, 32, false>(const KKTArgs&, hipStream_t);
}  // namespace noc
