// qpd_k_generic.hip -- the generic engine's kernel instantiations
// (generic_decode_kernel, qpd_generic.hip) as a translation unit of their own
// (build.py UNITS).
#include "qpd_generic.hip"
#include "qpd.h"

namespace qpd {

// Generic-engine instantiations generic_decode_kernel<family, domain>: every
// family in the LUT and plain float domains; the re-quantized domains exist
// only for SC and SCL (SC{,L}{Uniform,Lloyd}QuantizedDecoder).
const void *generic_kernel(int fam, int dom, bool wide) {
    using namespace qpd;
#define QPD_GK(K, D) (wide ? reinterpret_cast<const void *>(&generic_decode_kernel<K, D, kMaxLWide>) \
                           : reinterpret_cast<const void *>(&generic_decode_kernel<K, D, kMaxL>))
#define QPD_GN(K, D) reinterpret_cast<const void *>(&generic_decode_kernel<K, D, kMaxL>)
    // single-path families never need the wide list instantiation
    switch (dom) {
        case DOM_LUT:
            switch (fam) {
                case QPD_SC_LUT: return QPD_GN(K_SC_LUT, DOM_LUT);
                case QPD_SCL_LUT: return QPD_GK(K_SCL_LUT, DOM_LUT);
                case QPD_FASTSC_LUT: return QPD_GN(K_FASTSC_LUT, DOM_LUT);
                case QPD_FASTSCL_LUT: return QPD_GK(K_FASTSCL_LUT, DOM_LUT);
                default: return nullptr;
            }
        case DOM_FLOAT:
            switch (fam) {
                case QPD_SC_LUT: return QPD_GN(K_SC_LUT, DOM_FLOAT);
                case QPD_SCL_LUT: return QPD_GK(K_SCL_LUT, DOM_FLOAT);
                case QPD_FASTSC_LUT: return QPD_GN(K_FASTSC_LUT, DOM_FLOAT);
                case QPD_FASTSCL_LUT: return QPD_GK(K_FASTSCL_LUT, DOM_FLOAT);
                default: return nullptr;
            }
        case DOM_UNIFORM:
            return fam == QPD_SC_LUT ? QPD_GN(K_SC_LUT, DOM_UNIFORM)
                                     : fam == QPD_SCL_LUT ? QPD_GK(K_SCL_LUT, DOM_UNIFORM) : nullptr;
        case DOM_LLOYD:
            return fam == QPD_SC_LUT ? QPD_GN(K_SC_LUT, DOM_LLOYD)
                                     : fam == QPD_SCL_LUT ? QPD_GK(K_SCL_LUT, DOM_LLOYD) : nullptr;
        default: return nullptr;
    }
#undef QPD_GN
#undef QPD_GK
}

}  // namespace qpd
