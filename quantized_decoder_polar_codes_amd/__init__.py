"""MI355X-native quantized polar decoders (SC-LUT / SCL-LUT / FastSC-LUT /
FastSCL-LUT, CRC-aided CA-SCL-LUT / CA-FastSCL-LUT, plus float SC) behind the
reference's PolarDecoder class API.

Layout: ``csrc/`` holds the HIP kernels and the C-ABI (built in-tree into
``libqpd.so``); ``decoders`` mirrors the reference's pybind11 classes; ``codes``
and ``lut`` restate the host-side input producers (code construction, node
identification, LUT packing).
"""
from . import codes, lut  # noqa: F401
from .decoders import (  # noqa: F401
    CAFastSCLLUTDecoder,
    CASCLLUTDecoder,
    FastSCLLUTDecoder,
    FastSCLUTDecoder,
    SCDecoder,
    SCLLUTDecoder,
    SCLUTDecoder,
    from_packed,
)

__version__ = "0.1.0"
