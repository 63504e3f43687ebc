// Instantiation unit of the KKT scan for (nx, nu) = (4, 1), lanes 32 (see kkt_scan_4x1.hip).
#include "kkt_scan_impl.h"

namespace noc {
// the non-temporal phase-3 instances of large batches (kkt_nt3) live in a code object of their
// own (kkt_scan_4x1_l32nt.hip), so this unit's kernels keep the round-5 code object
extern template __global__ void kkt_scan_kernel<4, 1, 32, true, true, 0, false, true>(KKTArgs);
extern template __global__ void kkt_scan_kernel<4, 1, 32, false, true, 0, false, true>(KKTArgs);
template hipError_t launch_kkt<4, 1, 32, true>(const KKTArgs&, hipStream_t);
template hipError_t launch_kkt<4, 1, 32, false>(const KKTArgs&, hipStream_t);
}  // namespace noc
