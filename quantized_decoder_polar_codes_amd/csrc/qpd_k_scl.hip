// qpd_k_scl.hip -- SCL-LUT decode kernel instantiations with two pointer words
// per path (lut_fast_kernel<K_SCL_LUT, NS, L8>, qpd_fast.hip; see qpd_k_fast.hip);
// w16: list sizes 9..16 (W16, lane groups of 16).
#define QPD_FAST_TEMPLATES_ONLY
#include "qpd_fast.hip"
#include "qpd.h"

namespace qpd {

const void *fast_kernel_scl(int sets, bool l8, bool w16) {
#define QPD_FK(S, E) reinterpret_cast<const void *>(&lut_fast_kernel<K_SCL_LUT, S, E>)
#define QPD_FW(S) reinterpret_cast<const void *>(&lut_fast_kernel<K_SCL_LUT, S, false, false, false, false, true>)
    if (w16) return sets == 2 ? QPD_FW(2) : sets == 1 ? QPD_FW(1) : nullptr;
#ifdef QPD_SETS3
    if (sets == 3 && l8) return QPD_FK(3, true);
#endif
    if (sets == 2) return l8 ? QPD_FK(2, true) : QPD_FK(2, false);
    return l8 ? QPD_FK(1, true) : QPD_FK(1, false);
#undef QPD_FK
#undef QPD_FW
}

}  // namespace qpd
