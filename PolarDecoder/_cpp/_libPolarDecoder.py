"""Stands where the reference's extension module PolarDecoder._cpp._libPolarDecoder
(_libPolarDecoder.cpp:29-50) stood, for callers that import it directly."""
from quantized_decoder_polar_codes_amd.decoders import (  # noqa: F401
    CAFastSCLLUTDecoder,
    CASCLLUTDecoder,
    FastSCLLUTDecoder,
    FastSCLUTDecoder,
    SCDecoder,
    SCLLUTDecoder,
    SCLUTDecoder,
)
