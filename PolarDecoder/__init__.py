"""Drop-in replacement for the reference package ``PolarDecoder``
(/root/reference/PolarDecoder/PolarDecoder): same module paths and class names,
decoding on MI355X through libqpd.so.  All 15 classes: the LUT decoders of
the hot path (SC/SCL/FastSC/FastSCL-LUT), their CRC-aided variants
(CA-SCL-LUT, CA-FastSCL-LUT), and the float64-LLR decoders (SC, SCL, CA-SCL,
FastSC, FastSCL, SC/SCL uniform- and Lloyd-quantized)."""
from . import Decoder  # noqa: F401
from quantized_decoder_polar_codes_amd import __version__  # noqa: F401
