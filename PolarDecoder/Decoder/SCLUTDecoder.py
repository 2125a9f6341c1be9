from quantized_decoder_polar_codes_amd.decoders import SCLUTDecoder  # noqa: F401
