// classify4_cls instantiations other than the LDS-resident vector-load
// ones (k4_ldsv.hip), and the slot mode of connection batches.
#include "kernels_dev.hpp"

namespace cls {

hipError_t launch_classify4_cls(const Cls4Dev& t, const Pkts4& p, uint8_t* verdict,
                                unsigned long long* gslot, bool lds_resident, bool vec,
                                const LaunchCfg& cfg) {
    if (!cls_dispatchable(t, lds_resident, false)) return hipErrorInvalidValue;
    if (lds_resident) {
        if (vec) return launch_cls4_lds_vec(t, p, verdict, gslot, cfg);
        dispatch_cls<true, false>(t, p, verdict, gslot, cfg);
    } else {
        if (vec) dispatch_cls<false, true>(t, p, verdict, gslot, cfg);
        else dispatch_cls<false, false>(t, p, verdict, gslot, cfg);
    }
    return hipGetLastError();
}

hipError_t launch_classify4_slots(const Cls4Dev& t, const Pkts4& p, uint32_t* out, bool lds_resident,
                                  const LaunchCfg& cfg) {
    if (!cls_dispatchable(t, lds_resident, false)) return hipErrorInvalidValue;
    if (lds_resident) dispatch_slots4<true>(t, p, out, cfg);
    else dispatch_slots4<false>(t, p, out, cfg);
    return hipGetLastError();
}

}  // namespace cls
