#!/bin/bash
# Round 3 z3: SCL-LUT / CA-SCL-LUT at one frame set per wave (QPD_SETS=1, 6 waves
# per SIMD) vs the default two sets.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
: > $O/r03z3_sets.txt
for round in 1 2; do
  for kind in SCL-LUT CA-SCL-LUT; do
    for sets in 2 1; do
      QPD_SETS=$sets timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 4 --kind $kind > $O/r03z3_tmp.log 2>&1 || exit $?
      echo "$round sets=$sets $kind $(grep -o '"value": [0-9.]*' $O/r03z3_tmp.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $O/r03z3_tmp.log)" | tee -a $O/r03z3_sets.txt
    done
  done
done
echo done
