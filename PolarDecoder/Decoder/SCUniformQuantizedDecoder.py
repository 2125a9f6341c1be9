from quantized_decoder_polar_codes_amd.decoders import SCUniformQuantizedDecoder  # noqa: F401
