#!/bin/bash
# A/B: FastSCL-LUT with non-inlined special ops (build_variants/libqpd_noinl.so) at one and
# two frame sets, against the product build; SCL-LUT on both builds.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
: > $O/r03e_ab.txt
run() {  # tag env... -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 4 --kind $KIND > $O/r03e_tmp.log 2>&1 || return $?
  echo "$tag $KIND $(grep -o '"value": [0-9.]*' $O/r03e_tmp.log)" | tee -a $O/r03e_ab.txt
}
KIND=FastSCL-LUT
run head1 X=1 || exit $?
run noinl1 QPD_LIB=build_variants/libqpd_noinl.so || exit $?
run noinl2 QPD_LIB=build_variants/libqpd_noinl.so QPD_SETS=2 || exit $?
run head2 QPD_SETS=2 || exit $?
KIND=SCL-LUT
run head X=1 || exit $?
run noinl QPD_LIB=build_variants/libqpd_noinl.so || exit $?
