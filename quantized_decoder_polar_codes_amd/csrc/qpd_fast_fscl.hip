// qpd_fast_fscl.hip -- the FastSCL-LUT instantiations of lut_fast_kernel
// (qpd_fast.hip) with two pointer words per path.  The same kernel template as
// SCL-LUT -- two frame sets per wave, LDS byte tables, staged BOT3 loads,
// folded descents and combines -- with the special-node ops of
// FastSCLLUTDecoder.cpp:82-213 and the mixed bottom subtrees (botx_op)
// compiled in (KIND = K_FASTSCL_LUT).  See qpd_k_fast.hip for the units.
#define QPD_FAST_TEMPLATES_ONLY
#ifndef QPD_VEC_CHAIN  // lut_vec's results joined by one v_lshl_or each: FastSCL-LUT +0.5 %, SCL-LUT -0.25 % (r06v)
#define QPD_VEC_CHAIN 1
#endif
#include "qpd_fast.hip"

namespace qpd {

const void *fast_kernel_fscl(int sets, bool l8, bool r1l) {
#define QPD_F(S, E, R) reinterpret_cast<const void *>(&lut_fast_kernel<K_FASTSCL_LUT, S, E, R>)
    if (r1l) {
        if (sets == 2) return l8 ? QPD_F(2, true, true) : QPD_F(2, false, true);
        return l8 ? QPD_F(1, true, true) : QPD_F(1, false, true);
    }
    if (sets == 2) return l8 ? QPD_F(2, true, false) : QPD_F(2, false, false);
    return l8 ? QPD_F(1, true, false) : QPD_F(1, false, false);
#undef QPD_F
}

}  // namespace qpd
