from quantized_decoder_polar_codes_amd.decoders import FastSCLLUTDecoder  # noqa: F401
