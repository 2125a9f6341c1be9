// qpd_k_scl.hip -- SCL-LUT decode kernel instantiations with two pointer words
// per path (lut_fast_kernel<K_SCL_LUT, NS, L8>, qpd_fast.hip; see qpd_k_fast.hip).
#define QPD_FAST_TEMPLATES_ONLY
#include "qpd_fast.hip"
#include "qpd.h"

namespace qpd {

const void *fast_kernel_scl(int sets, bool l8) {
#define QPD_FK(S, E) reinterpret_cast<const void *>(&lut_fast_kernel<K_SCL_LUT, S, E>)
#ifdef QPD_SETS3
    if (sets == 3 && l8) return QPD_FK(3, true);
#endif
    if (sets == 2) return l8 ? QPD_FK(2, true) : QPD_FK(2, false);
    return l8 ? QPD_FK(1, true) : QPD_FK(1, false);
#undef QPD_FK
}

}  // namespace qpd
