from quantized_decoder_polar_codes_amd.decoders import SCLLloydQuantizedDecoder  # noqa: F401
