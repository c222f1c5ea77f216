// classify16_cls instantiations (16-byte layout) and their slot mode.
#include "kernels_dev.hpp"

namespace cls {

hipError_t launch_classify16_cls(const Cls4Dev& t, const Fe16& fe, const Pkts16& p, uint8_t* verdict,
                                 unsigned long long* gslot, bool lds_resident, bool lin,
                                 const LaunchCfg& cfg) {
    if (!lin && !cls_dispatchable(t, lds_resident, true)) return hipErrorInvalidValue;
    if (lds_resident) dispatch16<true>(t, fe, p, verdict, gslot, lin, cfg);
    else dispatch16<false>(t, fe, p, verdict, gslot, lin, cfg);
    return hipGetLastError();
}

hipError_t launch_classify16_slots(const Cls4Dev& t, const Fe16& fe, const Pkts16& p, uint32_t* out,
                                   bool lds_resident, const LaunchCfg& cfg) {
    if (!cls_dispatchable(t, lds_resident, true)) return hipErrorInvalidValue;
    if (lds_resident) dispatch_slots16<true>(t, fe, p, out, cfg);
    else dispatch_slots16<false>(t, fe, p, out, cfg);
    return hipGetLastError();
}

}  // namespace cls
