#!/bin/bash
# Code bytes of each decode kernel in one unit (default qpd_fast_fscl1.hip) with extra hipcc flags.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
U=qpd_fast_fscl1.hip
case "${1:-}" in *.hip) U=$1; shift;; esac
T=$(mktemp -d); cd $T
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include -I$ROOT/quantized_decoder_polar_codes_amd/csrc "$@" \
  -c $ROOT/quantized_decoder_polar_codes_amd/csrc/$U -o u.o -save-temps 2>/dev/null
/opt/rocm/lib/llvm/bin/llvm-readelf -s *gfx950.out | grep "FUNC.*lut_fast_kernel" | awk '{print $3, $8}' | sort -u
cd /; rm -rf $T
