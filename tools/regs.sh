#!/bin/bash
# Register / scratch / spill counts of one decode kernel unit (default: the
# FastSCL-LUT bench kernel, qpd_fast_fscl1.hip) with extra hipcc flags, in
# about 45 s -- the quick check before a full variant build.
# usage: tools/regs.sh [unit.hip] [-Dflags...]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
U=qpd_fast_fscl1.hip
case "${1:-}" in *.hip) U=$1; shift;; esac
T=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include -I$ROOT/quantized_decoder_polar_codes_amd/csrc "$@" \
  -c $ROOT/quantized_decoder_polar_codes_amd/csrc/$U -o $T/u.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -A12 "Function Name: _ZN3qpd15lut_fast_kernel" | grep -E "Function Name|VGPRs:|ScratchSize|VGPRs Spill|SGPRs Spill" \
  | sed 's/.*remark: //; s/\[-Rpass.*//' | paste - - - - - | sed "s/Function Name: _ZN3qpd15lut_fast_kernel/  /"
rm -rf $T
