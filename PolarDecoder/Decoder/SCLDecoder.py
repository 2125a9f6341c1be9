from quantized_decoder_polar_codes_amd.decoders import SCLDecoder  # noqa: F401
