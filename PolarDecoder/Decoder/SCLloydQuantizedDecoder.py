from quantized_decoder_polar_codes_amd.decoders import SCLloydQuantizedDecoder  # noqa: F401
