from quantized_decoder_polar_codes_amd.decoders import CAFastSCLLUTDecoder  # noqa: F401
