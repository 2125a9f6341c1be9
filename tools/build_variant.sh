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
UNITS=$(cd "$ROOT" && python3 -c "
from quantized_decoder_polar_codes_amd import build
for u, fl in build.UNITS: print(u + '|' + ' '.join(fl))")
# VARIANT_UNITS="a.hip b.hip": compile only those, link the rest from the last
# in-tree build (build/obj, build.py).  Refused when build/obj is not the current
# tree's build (its BUILD_ID), and for flags that change a struct the host unit
# fills (QPD_STAMPS adds FastPlan::stamps): then every unit must be rebuilt.
if [ -n "${VARIANT_UNITS:-}" ]; then
  case " $* " in *QPD_STAMPS*) echo "build_variant: VARIANT_UNITS with QPD_STAMPS changes FastPlan's layout; rebuild all units" >&2; exit 2;; esac
  want=$(cd "$ROOT" && python3 -c "from quantized_decoder_polar_codes_amd import build; print(build.source_hash())")
  have=$(cat "$ROOT/build/obj/BUILD_ID" 2>/dev/null || true)
  if [ "$want" != "$have" ] || [ -n "${QPD_VARIANT_SRC:-}" ]; then
    echo "build_variant: build/obj ($have) is not this tree's build ($want); run build.py or drop VARIANT_UNITS" >&2; exit 2
  fi
fi
objs=()
while IFS='|' read -r u fl; do
  o="$OUT/obj_$NAME/${u%.*}.o"
  [ -f "$SRC/$u" ] || continue
  if [ -n "${VARIANT_UNITS:-}" ] && [[ " $VARIANT_UNITS " != *" $u "* ]]; then
    objs+=("$ROOT/build/obj/${u%.*}.o"); continue
  fi
  $CXX $fl -c "$SRC/$u" -o "$o" -Rpass-analysis=kernel-resource-usage > "$OUT/obj_$NAME/${u%.*}.log" 2>&1 &
  objs+=("$o")
done <<< "$UNITS"
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$OUT/libqpd_$NAME.so"
cat "$OUT"/obj_$NAME/*.log | grep -A10 "Function Name: _ZN3qpd15lut_fast_kernel" \
  | grep -E "Function Name|VGPRs:|ScratchSize|SGPRs Spill" | sed 's/.*remark: //; s/\[-Rpass.*//' | paste - - - - \
  | sed "s/Function Name: _ZN3qpd15lut_fast_kernel/  /"
rm -rf "$OUT/obj_$NAME"
