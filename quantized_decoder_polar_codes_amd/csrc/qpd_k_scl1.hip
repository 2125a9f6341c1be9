// qpd_k_scl1.hip -- SCL-LUT decode kernel instantiations with one pointer word
// per path (lut_fast_kernel<K_SCL_LUT, NS, L8, false, false, PW1 = true>,
// qpd_fast.hip; see qpd_k_fast.hip).  The bench workload's kernel.
#define QPD_FAST_TEMPLATES_ONLY
#include "qpd_fast.hip"
#include "qpd.h"

namespace qpd {

const void *fast_kernel_scl_pw1(int sets, bool l8) {
#define QPD_FK(S, E) reinterpret_cast<const void *>(&lut_fast_kernel<K_SCL_LUT, S, E, false, false, true>)
    if (sets == 2) return l8 ? QPD_FK(2, true) : QPD_FK(2, false);
    if (sets == 1) return l8 ? QPD_FK(1, true) : QPD_FK(1, false);
    return nullptr;
#undef QPD_FK
}

}  // namespace qpd
