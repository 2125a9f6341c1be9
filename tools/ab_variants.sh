#!/bin/bash
# A/B of prebuilt variants (build_variants/libqpd_NAME.so), two alternating
# passes, after the GPU suite on the in-tree build.
# usage (GPU box, repo root): bash tools/ab_variants.sh "SCL-LUT FastSCL-LUT" NAME...
set -u
cd "$GRAFT_REPO_ROOT"
KINDS=$1; shift
mkdir -p gpurun_out
if [ -z "${AB_SKIP_TESTS:-}" ]; then
  timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
: > gpurun_out/ab.txt
for pass in 1 2; do
  for v in "$@"; do
    QPD_LIB=build_variants/libqpd_$v.so AB_TAG="$v" timeout -k 10 150 python tools/ab_kinds.py $KINDS >> gpurun_out/ab.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/ab.txt
