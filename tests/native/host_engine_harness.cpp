// Test harness (CPU): the host engine of libqpd.so (csrc/qpd_host.hpp) built
// with g++ beside the tests, so that its parity with the reference's golden
// vectors and the oracle is checked without a GPU.  The product reaches the
// same engine only through a device decoder (qpd_decode_host).
#include "qpd_host.hpp"

extern "C" int hh_decode(const qpd_config *c, const void *in, int64_t B, uint8_t *out) {
    std::unique_ptr<qpd_host::Plan> p = qpd_host::make_plan(c);
    if (!p) return -2;
    int flag = 0;
    if (p->dom == qpd::DOM_LUT) {
        qpd_host::Engine<uint8_t> e(*p);
        for (int64_t b = 0; b < B; ++b) flag |= e.decode((const int32_t *)in + b * p->N, out + b * p->out_k);
    } else {
        qpd_host::Engine<double> e(*p);
        for (int64_t b = 0; b < B; ++b) flag |= e.decode((const double *)in + b * p->N, out + b * p->out_k);
    }
    return flag;
}
