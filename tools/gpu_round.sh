#!/bin/bash
# Round record on the GPU box (repo root): rocprof kernel trace + PMC passes
# (tools/profile_round.sh), the HBM traffic record, the default bench line,
# and a per-op-class cycle breakdown (stamps build).  usage: bash tools/gpu_round.sh TAG
set -eu
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
bash tools/profile_round.sh "$TAG"
python tools/pmc_traffic.py SCL-LUT_N1024_K512_L8_F262144 gpurun_out/prof_$TAG/fetch/fetch_counter_collection.csv \
  gpurun_out/prof_$TAG/write/write_counter_collection.csv lut_fast_kernel,root_pre_kernel
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
grep -v amdgpu.ids gpurun_out/bench.log
if [ -f build_variants/libqpd_stampsd3.so ]; then
  STAMPS_DEPTH=1 QPD_LIB=build_variants/libqpd_stampsd3.so timeout -k 10 120 python tools/stamps.py SCL-LUT > gpurun_out/stamps_scl.txt 2>&1
  STAMPS_DEPTH=1 QPD_LIB=build_variants/libqpd_stampsd3.so timeout -k 10 120 python tools/stamps.py FastSCL-LUT > gpurun_out/stamps_fscl.txt 2>&1
fi
echo "round record $TAG done"
