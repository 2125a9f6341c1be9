#!/bin/bash
# One GPU session (run on the GPU box from the repo root): the GPU test suite on
# the in-tree build (TESTS=0 skips it, TESTS="expr" narrows it to -k expr), then A/B
# timings of prebuilt variants (build_variants/libqpd_NAME.so, tools/build_variant.sh)
# on the bench workload, two alternating passes.  Stops at the first crash,
# abort or time limit.
# usage: TAG=r05a KINDS="SCL-LUT FastSCL-LUT" bash tools/gpu_session.sh NAME[:VAR=VAL,...]...
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r05}
KINDS=${KINDS:-"SCL-LUT FastSCL-LUT"}
if [ "${TESTS:-1}" != "0" ]; then
  SEL=${TESTS:-1}
  [ "$SEL" = "1" ] && SEL=""  # TESTS="<pytest -k expression>"
  timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${SEL:+-k "$SEL"} \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?
  tail -4 gpurun_out/${TAG}_pytest.log
  # 0 passed, 1 test failures: timings still meaningful; anything else (crash, abort, limit): stop
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
[ $# -eq 0 ] && exit 0
: > gpurun_out/${TAG}_ab.txt
for pass in 1 2; do
  for spec in "$@"; do
    v=${spec%%:*}  # NAME or NAME:VAR=VAL,VAR=VAL (environment of that run)
    envs=""
    [ "$spec" != "$v" ] && envs=${spec#*:} && envs=${envs//,/ }
    lib=build_variants/libqpd_$v.so
    [ "$v" = "tree" ] && lib=quantized_decoder_polar_codes_amd/libqpd.so
    env $envs QPD_LIB=$lib AB_TAG="$spec" timeout -k 10 200 python tools/ab_kinds.py $KINDS >> gpurun_out/${TAG}_ab.txt 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then grep -v amdgpu.ids gpurun_out/${TAG}_ab.txt | tail -20; echo "ab rc=$rc ($v): stopping"; exit $rc; fi
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}_ab.txt
