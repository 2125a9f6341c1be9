// Test infrastructure only (oracle/_ref): a pybind11 module definition that
// exposes the reference decoders compiled from their own sources under
// /root/reference/PolarDecoder/PolarDecoder/_cpp.  It replaces the reference's
// _libPolarDecoder.cpp (_libPolarDecoder.cpp:29-50) only to skip
// NDArrayConverter::init_numpy(), which needs OpenCV and is unused by the
// decoders.  Nothing here is shipped or measured as the product.
#include <pybind11/pybind11.h>
namespace py = pybind11;

void init_SCDecoder(py::module &m);
void init_SCLUTDecoder(py::module &m);
void init_SCLLUTDecoder(py::module &m);
void init_FastSCLUTDecoder(py::module &m);
void init_FastSCLLUTDecoder(py::module &m);
void init_CASCLLUTDecoder(py::module &m);
void init_CAFastSCLLUTDecoder(py::module &m);
void init_SCLDecoder(py::module &m);
void init_CASCLDecoder(py::module &m);
void init_FastSCDecoder(py::module &m);
void init_FastSCLDecoder(py::module &m);
void init_SCUniformQuantizedDecoder(py::module &m);
void init_SCLUniformQuantizedDecoder(py::module &m);
void init_SCLloydQuantizedDecoder(py::module &m);
void init_SCLLloydQuantizedDecoder(py::module &m);

PYBIND11_MODULE(_refPolarDecoder, m) {
    m.doc() = "reference decoders (oracle build, test-only)";
    init_SCDecoder(m);
    init_SCLUTDecoder(m);
    init_SCLLUTDecoder(m);
    init_FastSCLUTDecoder(m);
    init_FastSCLLUTDecoder(m);
    init_CASCLLUTDecoder(m);
    init_CAFastSCLLUTDecoder(m);
    init_SCLDecoder(m);
    init_CASCLDecoder(m);
    init_FastSCDecoder(m);
    init_FastSCLDecoder(m);
    init_SCUniformQuantizedDecoder(m);
    init_SCLUniformQuantizedDecoder(m);
    init_SCLloydQuantizedDecoder(m);
    init_SCLLloydQuantizedDecoder(m);
}
