"""Drop-in replacement for the reference package ``PolarDecoder``
(/root/reference/PolarDecoder/PolarDecoder): same module paths and class names,
decoding on MI355X through libqpd.so.  Only the LUT decoders of the hot path
and the float SC decoder are provided."""
from . import Decoder  # noqa: F401
from quantized_decoder_polar_codes_amd import __version__  # noqa: F401
