# Same shape as the reference (PolarDecoder/PolarDecoder/Decoder/__init__.py:1-3):
# the submodules are imported, each holding its class of the same name.
from . import (  # noqa: F401
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
