// Instantiation unit of the KKT scan for (nx, nu) = (4, 1), lanes 64 / 16 / 8; see kkt_scan_impl.h.
// Lanes 32 (c3) and 128 (the two-wave segments) are compiled in parallel units
// (kkt_scan_4x1_l32.hip, kkt_scan_4x1_l128.hip): shorter builds, and each hot instance in a code
// object of its own (the 512 shard's byte-identical L = 128 kernel ran 3 % slower when the
// unit's other kernels grew, profiles/r05/ab_slots/).
#include "kkt_scan_impl.h"

namespace noc {
#ifndef NOC_SCAN_STAMPS  // the stamps build keeps every instance here: one g_scan_stamps table
extern template hipError_t launch_kkt<4, 1, 32, true>(const KKTArgs&, hipStream_t);
extern template hipError_t launch_kkt<4, 1, 32, false>(const KKTArgs&, hipStream_t);
extern template hipError_t launch_kkt<4, 1, 128, true>(const KKTArgs&, hipStream_t);
extern template hipError_t launch_kkt<4, 1, 128, false>(const KKTArgs&, hipStream_t);
#endif

template <>
hipError_t kkt_dispatch_shape<4, 1>(const KKTArgs& a, int lanes, hipStream_t stream) {
  return dispatch_aff<4, 1>(a, lanes, stream);
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
