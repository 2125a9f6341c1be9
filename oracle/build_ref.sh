#!/usr/bin/env bash
# Build the reference decoders (test oracle only) from their sources where they
# lie under /root/reference.  Output goes to oracle/_ref/ (git-ignored).  The
# GPU box has no /root/reference; it uses the prebuilt .so if present.
# Flags mirror the reference's Release build (PolarDecoder/CMakeLists.txt:5,8,17:
# -O3, -DNDEBUG) so the compiled-out asserts and libstdc++ std::sort behave
# exactly as in the reference.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
R=/root/reference/PolarDecoder/PolarDecoder/_cpp
if [ ! -d "$R" ]; then
  echo "build_ref: $R absent; skipping reference build" >&2
  exit 0
fi
OUT="$HERE/_ref"
mkdir -p "$OUT"
SUFFIX="$(python3-config --extension-suffix)"
TARGET="$OUT/_refPolarDecoder$SUFFIX"
SRCS="utils SCDecoder SCLUTDecoder SCLLUTDecoder FastSCLUT FastSCLLUTDecoder CASCLLUTDecoder CAFastSCLLUTDecoder
      SCLDecoder CASCLDecoder FastSCDecoder FastSCLDecoder SCUniformQuantizedDecoder SCLUniformQuantizedDecoder
      SCLloydQuantizedDecoder SCLLloydQuantizedDecoder"
PYI="py_SCDecoder py_SCLUTDecoder py_SCLLUTDecoder py_FastSCLUTDecoder py_FastSCLLUTDecoder py_CASCLLUTDecoder py_CAFastSCLLUTDecoder
     py_SCLDecoder py_CASCLDecoder py_FastSCDecoder py_FastSCLDecoder py_SCUniformDecoder py_SCLUniformQuantizedDecoder
     py_SCLloydQuantizedDecoder py_SCLLloydQuantizedDecoder"
FILES=""
for s in $SRCS; do FILES="$FILES $R/src/$s.cpp"; done
for s in $PYI; do FILES="$FILES $R/py_interface/$s.cpp"; done
NEWEST=0
if [ -f "$TARGET" ] && [ "$TARGET" -nt "$HERE/ref_module.cpp" ]; then
  echo "build_ref: up to date: $TARGET"
  exit 0
fi
OBJDIR="$OUT/obj"; mkdir -p "$OBJDIR"
INC="-I$R/include $(python3 -m pybind11 --includes)"
CXXFLAGS="-O3 -DNDEBUG -std=c++11 -fPIC -w"
pids=()
objs=()
for f in $FILES "$HERE/ref_module.cpp"; do
  o="$OBJDIR/$(basename "$f" .cpp).o"
  objs+=("$o")
  g++ $CXXFLAGS $INC -c "$f" -o "$o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
g++ -shared -o "$TARGET" "${objs[@]}"
echo "build_ref: built $TARGET"
