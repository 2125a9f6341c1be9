from quantized_decoder_polar_codes_amd.decoders import FastSCDecoder  # noqa: F401
