// qpd_fast_fscl1.hip -- the FastSCL-LUT decode kernel with one pointer word per
// path, two frame sets and L = 8 (lut_fast_kernel<K_FASTSCL_LUT, 2, true, false,
// false, true>, qpd_fast.hip): the config-C4 bench kernel.  See qpd_k_fast.hip.
#define QPD_FAST_TEMPLATES_ONLY
#ifndef QPD_VEC_CHAIN  // lut_vec's results joined by one v_lshl_or each: FastSCL-LUT +0.5 %, SCL-LUT -0.25 % (r06v)
#define QPD_VEC_CHAIN 1
#endif
#include "qpd_fast.hip"

namespace qpd {

const void *fast_kernel_fscl_pw1(int sets, bool l8, bool r1l) {
    if (sets != 2 || !l8 || r1l) return nullptr;
    return reinterpret_cast<const void *>(&lut_fast_kernel<K_FASTSCL_LUT, 2, true, false, false, true>);
}

}  // namespace qpd
