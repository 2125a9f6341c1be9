// qpd_k_scl1.hip -- SCL-LUT decode kernel instantiations with one pointer word
// per path (lut_fast_kernel<K_SCL_LUT, NS, L8, false, false, PW1 = true>,
// qpd_fast.hip; see qpd_k_fast.hip).  The bench workload's kernel; w16: list sizes
// 9..16 (W16).
#define QPD_FAST_TEMPLATES_ONLY
#include "qpd_fast.hip"
#include "qpd.h"

namespace qpd {

const void *fast_kernel_scl_pw1(int sets, bool l8, bool w16) {
#define QPD_FK(S, E) reinterpret_cast<const void *>(&lut_fast_kernel<K_SCL_LUT, S, E, false, false, true>)
#define QPD_FW(S) reinterpret_cast<const void *>(&lut_fast_kernel<K_SCL_LUT, S, false, false, false, true, true>)
    if (w16) return sets == 2 ? QPD_FW(2) : sets == 1 ? QPD_FW(1) : nullptr;
    if (sets == 2) return l8 ? QPD_FK(2, true) : QPD_FK(2, false);
    if (sets == 1) return l8 ? QPD_FK(1, true) : QPD_FK(1, false);
    return nullptr;
#undef QPD_FK
#undef QPD_FW
}

}  // namespace qpd
