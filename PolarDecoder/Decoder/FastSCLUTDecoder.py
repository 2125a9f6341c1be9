from quantized_decoder_polar_codes_amd.decoders import FastSCLUTDecoder  # noqa: F401
