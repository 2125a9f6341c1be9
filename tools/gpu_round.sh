#!/bin/bash
# Round record on the GPU box (repo root): rocprof kernel trace + PMC passes
# folded into profiles/counters.json (tools/profile_round.sh), the default
# bench line, and a per-op-class cycle breakdown (stamps build, if built).
# usage: bash tools/gpu_round.sh TAG
set -eu
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
bash tools/profile_round.sh "$TAG"
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1
grep -v amdgpu.ids gpurun_out/bench_$TAG.log
if [ -f build_variants/libqpd_stampsd3.so ]; then
  STAMPS_DEPTH=1 QPD_LIB=build_variants/libqpd_stampsd3.so timeout -k 10 120 python tools/stamps.py SCL-LUT > gpurun_out/stamps_scl.txt 2>&1
  STAMPS_DEPTH=1 QPD_LIB=build_variants/libqpd_stampsd3.so timeout -k 10 120 python tools/stamps.py FastSCL-LUT > gpurun_out/stamps_fscl.txt 2>&1
fi
echo "round record $TAG done"
