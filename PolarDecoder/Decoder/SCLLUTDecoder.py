from quantized_decoder_polar_codes_amd.decoders import SCLLUTDecoder  # noqa: F401
