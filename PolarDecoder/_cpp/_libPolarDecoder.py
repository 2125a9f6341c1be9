"""Stands where the reference's extension module PolarDecoder._cpp._libPolarDecoder
(_libPolarDecoder.cpp:29-50) stood, for callers that import it directly: all
15 classes."""
from quantized_decoder_polar_codes_amd.decoders import (  # noqa: F401
    CAFastSCLLUTDecoder,
    CASCLDecoder,
    CASCLLUTDecoder,
    FastSCDecoder,
    FastSCLDecoder,
    FastSCLLUTDecoder,
    FastSCLUTDecoder,
    SCDecoder,
    SCLDecoder,
    SCLLUTDecoder,
    SCLLloydQuantizedDecoder,
    SCLUTDecoder,
    SCLUniformQuantizedDecoder,
    SCLloydQuantizedDecoder,
    SCUniformQuantizedDecoder,
)
