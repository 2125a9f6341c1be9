#!/bin/bash
# usage: tools/build_variant.sh NAME [extra hipcc flags...] -> build_variants/libqpd_NAME.so
# (A/B builds for tools/sweep.py via QPD_LIB=...; prints the fast kernels' resource usage.)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$ROOT/build_variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I"$ROOT/include" \
  -I"$ROOT/quantized_decoder_polar_codes_amd/csrc" "$@" "$ROOT/quantized_decoder_polar_codes_amd/csrc/qpd_capi.hip" "$ROOT/quantized_decoder_polar_codes_amd/csrc/qpd_fast_fscl.hip" "$ROOT/quantized_decoder_polar_codes_amd/csrc/qpd_lutgen.cpp" \
  -o "$ROOT/build_variants/libqpd_$NAME.so" -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -A8 "lut_fast_kernel" | grep -E "Function Name|VGPRs:|ScratchSize" \
  | sed 's/.*remark: //; s/\[-Rpass.*//' | paste - - - | sed "s/Function Name: _ZN3qpd15lut_fast_kernel/  /"
