#!/bin/bash
# A/B of two builds (build_variants/libqpd_<A>.so, _<B>.so), interleaved twice.
# usage (GPU box, repo root): bash tools/ab_pair.sh A B [kinds...]
set -u
cd "$GRAFT_REPO_ROOT"
A=$1; B=$2; shift 2
KINDS=${*:-SCL-LUT FastSCL-LUT CA-SCL-LUT}
: > gpurun_out/ab_pair.txt
for v in $A $B $A $B; do
  QPD_LIB=build_variants/libqpd_$v.so AB_TAG=$v timeout -k 10 150 python tools/ab_kinds.py $KINDS >> gpurun_out/ab_pair.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/ab_pair.txt
