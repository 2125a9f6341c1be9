from quantized_decoder_polar_codes_amd.decoders import CASCLDecoder  # noqa: F401
