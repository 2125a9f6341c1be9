#!/bin/bash
# usage: tools/build_variant.sh NAME [extra hipcc flags...] -> build_variants/libqpd_NAME.so
# A/B builds (QPD_LIB=build_variants/libqpd_NAME.so): the product's units and
# per-unit flags (build.py UNITS), compiled in parallel, plus the extra flags;
# prints the fast kernels' register / scratch usage.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT="$ROOT/build_variants"
mkdir -p "$OUT/obj_$NAME"
SRC="${QPD_VARIANT_SRC:-$ROOT/quantized_decoder_polar_codes_amd/csrc}"  # another tree: QPD_VARIANT_SRC=DIR/csrc
CXX="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I${QPD_VARIANT_INC:-$ROOT/include} -I$SRC $*"
$CXX -c "$SRC/qpd_capi.hip" -o "$OUT/obj_$NAME/capi.o" -Rpass-analysis=kernel-resource-usage > "$OUT/obj_$NAME/capi.log" 2>&1 &
$CXX -mllvm -amdgpu-sched-strategy=${FSCL_SCHED:-max-ilp} -c "$SRC/qpd_fast_fscl.hip" -o "$OUT/obj_$NAME/fscl.o" -Rpass-analysis=kernel-resource-usage > "$OUT/obj_$NAME/fscl.log" 2>&1 &
$CXX -c "$SRC/qpd_lutgen.cpp" -o "$OUT/obj_$NAME/lutgen.o" > "$OUT/obj_$NAME/lutgen.log" 2>&1 &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$OUT/obj_$NAME/capi.o" "$OUT/obj_$NAME/fscl.o" "$OUT/obj_$NAME/lutgen.o" -o "$OUT/libqpd_$NAME.so"
cat "$OUT/obj_$NAME/capi.log" "$OUT/obj_$NAME/fscl.log" | grep -A10 "Function Name: _ZN3qpd15lut_fast_kernel" \
  | grep -E "Function Name|VGPRs:|ScratchSize|SGPRs Spill" | sed 's/.*remark: //; s/\[-Rpass.*//' | paste - - - - \
  | sed "s/Function Name: _ZN3qpd15lut_fast_kernel/  /"
rm -rf "$OUT/obj_$NAME"
