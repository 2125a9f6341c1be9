// qpd_fast_fscl.hip -- the FastSCL-LUT instantiations of lut_fast_kernel
// (qpd_fast.hip), compiled as their own translation unit so that build.py can
// give them the max-ILP machine scheduler (-amdgpu-sched-strategy=max-ilp):
// on the bench workload it makes FastSCL-LUT 30.0 -> 31.5 M frames/s and
// SCL-LUT 0.5 % slower, with the same output digests (profiles/r02f_ab_ilp.txt),
// so only FastSCL takes it.  Diagnostic builds that read device globals
// (QPD_STAMPS) keep every instantiation in qpd_capi.hip instead.
// The kernel templates come from qpd_fast_fscl_kernel.hip (qpd::fscl), the
// FastSCL-LUT copy of the decode kernel (see there why).
#define QPD_FAST_TEMPLATES_ONLY
#define QPD_LANE_READ_SHFL  // HIP's __shfl for the shuffles (see lane_read, qpd_common.hpp)
#include "qpd_fast_fscl_kernel.hip"

namespace qpd {

const void *fast_kernel_fscl(int sets, bool l8, bool r1l) {
#define QPD_F(S, E, R) reinterpret_cast<const void *>(&fscl::lut_fast_kernel<K_FASTSCL_LUT, S, E, R>)
    if (r1l) {
        if (sets == 2) return l8 ? QPD_F(2, true, true) : QPD_F(2, false, true);
        return l8 ? QPD_F(1, true, true) : QPD_F(1, false, true);
    }
    if (sets == 2) return l8 ? QPD_F(2, true, false) : QPD_F(2, false, false);
    return l8 ? QPD_F(1, true, false) : QPD_F(1, false, false);
#undef QPD_F
}

}  // namespace qpd
