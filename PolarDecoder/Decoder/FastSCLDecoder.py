from quantized_decoder_polar_codes_amd.decoders import FastSCLDecoder  # noqa: F401
