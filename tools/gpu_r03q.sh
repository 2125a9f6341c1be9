#!/bin/bash
# Round 3 q: FastSCL-LUT register-allocation variants (AMDGPU trackers; 5 waves
# per SIMD; both) against the product build, two interleaved rounds.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
: > $O/r03q_ab.txt
for round in 1 2; do
  for lib in prod trk w5 w5trk; do
    if [ $lib = prod ]; then unset QPD_LIB; else export QPD_LIB=build_variants/libqpd_$lib.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 4 --kind FastSCL-LUT > $O/r03q_tmp.log 2>&1 || exit $?
    echo "$round $lib $(grep -o '"value": [0-9.]*' $O/r03q_tmp.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $O/r03q_tmp.log)" | tee -a $O/r03q_ab.txt
  done
done
echo done
