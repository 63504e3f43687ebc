// Instantiation unit of the KKT scan for (nx, nu) = (2, 1); see kkt_scan_impl.h.
#include "kkt_scan_impl.h"

namespace noc {
template <>
hipError_t kkt_dispatch_shape<2, 1>(const KKTArgs& a, int lanes, hipStream_t stream) {
  return dispatch_aff<2, 1>(a, lanes, stream);
}
}  // namespace noc

#ifdef NOC_SCAN_STAMPS
// diagnostic export of the stamps build (not part of the ABI header): copies waves x 8 x 2
// stamps (realtime, shader clock) of the last launches and zeroes the table when reset != 0
extern "C" int noc_debug_scan_stamps(long long* out, int waves, int reset) {
  if (waves > noc::kStampWaves) waves = noc::kStampWaves;
  const size_t bytes = (size_t)waves * noc::kStampSlots * 2 * sizeof(long long);
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(noc::g_scan_stamps), bytes) != hipSuccess) return -1;
  if (reset) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(noc::g_scan_stamps)) != hipSuccess) return -1;
    if (hipMemset(p, 0, sizeof(noc::g_scan_stamps)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
