from quantized_decoder_polar_codes_amd.decoders import SCDecoder  # noqa: F401
