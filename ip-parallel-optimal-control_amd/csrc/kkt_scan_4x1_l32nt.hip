// Instantiation unit of the KKT scan for (nx, nu) = (4, 1), lanes 32: the instances whose phase 3
// reads Q, R, M, r, q non-temporally (batches beyond 1.5x the memory-side cache, kkt_nt3).
#include "kkt_scan_impl.h"

namespace noc {
template __global__ void kkt_scan_kernel<4, 1, 32, true, true, 0, false, true>(KKTArgs);
template __global__ void kkt_scan_kernel<4, 1, 32, false, true, 0, false, true>(KKTArgs);
}  // namespace noc
