// classify4_cls instantiations: LDS-resident image, vector loads (the hot
// path; specialised on the sublist search depth).
#include "kernels_dev.hpp"

namespace cls {

hipError_t launch_cls4_lds_vec(const Cls4Dev& t, const Pkts4& p, uint8_t* verdict, unsigned long long* gslot,
                               const LaunchCfg& cfg) {
    dispatch_cls<true, true>(t, p, verdict, gslot, cfg);
    return hipGetLastError();
}

}  // namespace cls
