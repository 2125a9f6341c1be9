from quantized_decoder_polar_codes_amd.decoders import CASCLLUTDecoder  # noqa: F401
