#!/bin/bash
# Round record on the GPU box (repo root), stopping at the first failure:
# the GPU suite, smoke(), rocprofv3 kernel stats + PMC passes of the SCL-LUT
# and FastSCL-LUT bench workloads (tools/profile_round.sh -> profiles/counters.json,
# which the bench lines read), the default bench line (SCL-LUT, the headline),
# the FastSCL-LUT line (config C4) and config C5's 10^8-frame point.
# usage: bash tools/gpu_record.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r05}
mkdir -p gpurun_out
step() {  # name command...
  local name=$1; shift
  "$@" > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?
  echo "[$name rc=$rc]"; grep -v amdgpu.ids gpurun_out/${TAG}_$name.log | tail -3
  [ $rc -eq 0 ] || exit $rc
}
step pytest timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step prof_scl bash tools/profile_round.sh ${TAG}_scl --kind SCL-LUT
step prof_fscl bash tools/profile_round.sh ${TAG}_fscl --kind FastSCL-LUT
step bench timeout -k 10 300 python bench.py
step bench_fscl timeout -k 10 300 python bench.py --kind FastSCL-LUT
step mc timeout -k 10 300 python bench.py --mc-frames 1e8 --no-cpu-baseline
# the fast engine's lane groups of 16 (SCL-LUT at L = 16) and BASELINE config C2
step bench_l16 timeout -k 10 300 python bench.py --L 16 --frames 1048576 --no-e2e
step bench_c2 timeout -k 10 300 python bench.py --kind SC-LUT --N 128 --K 32 --frames 16777216 --no-e2e
echo "record $TAG done"
