#!/bin/bash
# GPU session: the GPU test suite, then A/B timings of the schedule variants
# (env switches) and of a reference build (QPD_LIB) on the bench workload.
# usage (GPU box, repo root): bash tools/gpu_ab.sh [reference .so] [env configs...]
set -u
cd "$GRAFT_REPO_ROOT"
REF=${1:-build_variants/libqpd_head.so}
shift || true
CFGS=("$@")
[ ${#CFGS[@]} -eq 0 ] && CFGS=("X=1" "QPD_NO_PRE=1" "QPD_NO_BFUSE=1")
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
: > gpurun_out/ab.txt
for cfg in "${CFGS[@]}"; do
  env $cfg AB_TAG="new $cfg" timeout -k 10 150 python tools/ab_kinds.py SCL-LUT FastSCL-LUT CA-SCL-LUT >> gpurun_out/ab.txt 2>&1 || exit $?
done
QPD_LIB=$REF timeout -k 10 150 python tools/ab_kinds.py SCL-LUT FastSCL-LUT CA-SCL-LUT >> gpurun_out/ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/ab.txt
