// qpd_k_fast.hip -- decode kernel instantiations (lut_fast_kernel, qpd_fast.hip)
// of SC-LUT and FastSC-LUT, and the frozen-prefix stages' (lut_prefix_kernel).
// The instantiations are spread over several translation units (this one,
// qpd_k_scl.hip, qpd_k_scl1.hip, qpd_fast_fscl.hip, qpd_fast_fscl1.hip; build.py
// UNITS) that compile in parallel.  nullptr for a combination that has no
// instantiation, so the launch fails loudly.
#define QPD_FAST_TEMPLATES_ONLY
#include "qpd_fast.hip"
#include "qpd.h"

namespace qpd {

const void *fast_kernel_single(int kind, int sets) {
#define QPD_FK(K, S) reinterpret_cast<const void *>(&lut_fast_kernel<K, S, false>)
    switch (kind) {
        case QPD_SC_LUT: return sets == 2 ? QPD_FK(K_SC_LUT, 2) : QPD_FK(K_SC_LUT, 1);
        case QPD_FASTSC_LUT: return sets == 2 ? QPD_FK(K_FASTSC_LUT, 2) : QPD_FK(K_FASTSC_LUT, 1);
        default: return nullptr;
    }
#undef QPD_FK
}

const void *prefix_kernel(int kind, int sets, bool pw1) {
    if (kind != QPD_SCL_LUT) return nullptr;
    if (pw1)
        return sets == 2 ? reinterpret_cast<const void *>(&lut_prefix_kernel(K_SCL_LUT, 2, true))
                         : reinterpret_cast<const void *>(&lut_prefix_kernel(K_SCL_LUT, 1, true));
    return sets == 2 ? reinterpret_cast<const void *>(&lut_prefix_kernel(K_SCL_LUT, 2, false))
                     : reinterpret_cast<const void *>(&lut_prefix_kernel(K_SCL_LUT, 1, false));
}

}  // namespace qpd
