from quantized_decoder_polar_codes_amd.decoders import SCLUniformQuantizedDecoder  # noqa: F401
